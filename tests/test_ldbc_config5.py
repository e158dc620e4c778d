"""Config 5 on the reference's LDBC sample (199 KNOWS edges among 88 persons):
var-length expand *1..3 (VarLengthExpandPlanner.scala:82-259) + DISTINCT +
two GROUP BY stages.  Oracle pinned by an independent brute-force path walk
(relationship-isomorphic paths: no edge repeated within a path)."""
import json
import os
from collections import Counter, defaultdict

import pytest

from ldbc import config5_query, ldbc_graph_data

from capf_amd.graph import ScanGraph
from capf_amd.planner import run
from oracle.table_np import OracleSession

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def brute_force(upper=3):
    g = ldbc_graph_data()
    persons = {n[0] for n in g.nodes}
    out = defaultdict(list)
    for rid, s, t, _, _ in g.rels:
        out[s].append((rid, t))
    reach = defaultdict(set)

    def walk(a, v, used, depth):
        for rid, t in out[v]:
            if rid in used:
                continue
            if t in persons:
                reach[a].add(t)
            if depth + 1 < upper:
                walk(a, t, used | {rid}, depth + 1)

    for a in persons:
        walk(a, a, frozenset(), 0)
    hist = Counter(len(bs) for bs in reach.values() if bs)
    return sorted([k, v] for k, v in hist.items())


def test_config5_oracle_vs_brute_force():
    got = run(ScanGraph.from_data(OracleSession(), ldbc_graph_data()), config5_query())
    assert sorted([r["reach"], r["n"]] for r in got) == brute_force()


def test_config5_golden_fixture():
    with open(os.path.join(HERE, "rmat_counts.json")) as f:
        assert json.load(f)["ldbc_config5"] == brute_force()


@pytest.mark.gpu
def test_config5_gpu(gpu_session):
    got = run(ScanGraph.from_data(gpu_session, ldbc_graph_data()), config5_query())
    assert sorted([r["reach"], r["n"]] for r in got) == brute_force()
