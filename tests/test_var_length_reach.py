"""Fused config-5 path (csrc/var_length_reach.hip via planner._fused_reach):
VarLengthExpand *1..u → DISTINCT (a, b) → GROUP BY a count(*) on the GPU,
against (1) the scipy matrix-power restatement (oracle/reach.py), (2) the
unfused relational plan on the GPU (CAPF_FUSED_REACH=0: join chain +
isomorphism filters + UNION ALL + DISTINCT + GROUP BY) and (3) the
isomorphic-path brute force on the reference's LDBC sample."""
import numpy as np
import pytest

from ldbc import config5_query, ldbc_graph_data

from capf_amd.expr import CountStar, Var
from capf_amd.graph import GraphData, ScanGraph
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run
from oracle import cmodel
from oracle import reach as oreach


def synthetic(scale, person_frac=0.6, seed=5):
    """R-MAT edges on sparse LDBC-style ids, Person/Other labels, KNOWS plus
    a second rel type that the pattern must ignore."""
    src, dst = cmodel.rmat(scale)
    n = 1 << scale
    rng = np.random.default_rng(seed)
    ids = np.arange(n, dtype=np.int64) * 1000003 + 65 - (n // 2) * 1000003  # negatives too
    person = rng.random(n) < person_frac
    nodes = [(int(ids[i]), frozenset(["Person" if person[i] else "Other"]), {}) for i in range(n)]
    other = rng.random(len(src)) < 0.1
    rels = [(10 ** 12 + k, int(ids[s]), int(ids[d]), "LIKES" if other[k] else "KNOWS", {})
            for k, (s, d) in enumerate(zip(src.tolist(), dst.tolist()))]
    knows = ~other
    return (GraphData(nodes, rels), ids[src[knows]], ids[dst[knows]], ids[person])


def reach_query(upper, direction="out"):
    return Query([Match([NodeP("a", ("Person",)), NodeP("b", ("Person",))],
                        [RelP("k", "a", "b", ("KNOWS",), direction=direction, length=(1, upper))])],
                 [Stage([("a", Var("a")), ("b", Var("b"))], distinct=True),
                  Stage([("a", Var("a")), ("reach", CountStar())])])


def test_oracle_on_ldbc_sample():
    g = ldbc_graph_data()
    src = np.array([r[1] for r in g.rels])
    dst = np.array([r[2] for r in g.rels])
    persons = np.array([nd[0] for nd in g.nodes])
    from test_ldbc_config5 import brute_force
    assert oreach.config5_histogram(src, dst, persons, persons) == brute_force()


@pytest.mark.gpu
def test_config5_fused_on_ldbc_sample(gpu_session):
    from test_ldbc_config5 import brute_force
    g = ScanGraph.from_data(gpu_session, ldbc_graph_data())
    got = run(g, config5_query())
    assert sorted([r["reach"], r["n"]] for r in got) == brute_force()


@pytest.mark.gpu
@pytest.mark.parametrize("upper", [1, 2, 3, 4])
@pytest.mark.parametrize("compact", [False, True], ids=["int64", "for32"])
def test_reach_vs_matrix_powers(gpu_session, upper, compact):
    data, ks, kd, persons = synthetic(10)
    g = ScanGraph.from_data(gpu_session, data, compact=compact)
    got = {r["a"]: r["reach"] for r in run(g, reach_query(upper))}
    assert got == oreach.reach_counts(ks, kd, persons, persons, upper)


@pytest.mark.gpu
def test_reach_incoming_direction(gpu_session):
    data, ks, kd, persons = synthetic(9)
    g = ScanGraph.from_data(gpu_session, data)
    # (a)<-[:KNOWS*1..3]-(b) grouped by b: walks from b along the rels
    q = Query([Match([NodeP("a", ("Person",)), NodeP("b", ("Person",))],
                     [RelP("k", "a", "b", ("KNOWS",), direction="in", length=(1, 3))])],
              [Stage([("a", Var("a")), ("b", Var("b"))], distinct=True),
               Stage([("b", Var("b")), ("reach", CountStar())])])
    got = {r["b"]: r["reach"] for r in run(g, q)}
    assert got == oreach.reach_counts(ks, kd, persons, persons, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("upper", [2, 3])
def test_fused_equals_relational_plan(gpu_session, monkeypatch, upper):
    """The fused operator and the okapi relational lowering (join chain with
    relationship-isomorphism filters, UNION ALL, DISTINCT, GROUP BY) agree
    row for row on the GPU, self-loops and multi-edges included."""
    data, *_ = synthetic(6)
    g = ScanGraph.from_data(gpu_session, data)
    q = reach_query(upper)
    q.stages.append(Stage([("reach", Var("reach")), ("n", CountStar())]))
    fused = sorted([r["reach"], r["n"]] for r in run(g, q))
    monkeypatch.setenv("CAPF_FUSED_REACH", "0")
    plain = sorted([r["reach"], r["n"]] for r in run(g, q))
    assert fused == plain
