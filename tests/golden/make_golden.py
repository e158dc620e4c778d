"""Generates the committed golden fixtures (run from the repo root in the dev
container; /root/reference is only read here, never at test time):

  reference_cases.json  expected Bags of the reference acceptance tests
                        (transcribed in reference_cases.py) + the oracle's Bags
  ldbc_sample.json      the reference's LDBC sample KNOWS graph
                        (morpheus-examples/src/main/resources/ldbc/csv/
                        person_0_0.csv.gz, person_knows_person_0_0.csv.gz)
  config5_sf10.json     config 5 at its BASELINE size (2^16 Person, R-MAT edge
                        factor 30): the RETURN reach, count(*) histogram by
                        the C bitset BFS (oracle/rmat.c::reach_bitset)
  rmat_counts.json      R-MAT counts of configs 2/3 at small scales by the
                        closed forms (oracle/rmat.c), plus the config-5 query
                        on the LDBC sample by the oracle table;
                        "full": configs 2/3 at the headline sizes (s20-s24,
                        streamed closed forms, rmat_stream_counts);
                        "triangle": config 4 by trace(A^3) intersection
                        (count_triangle_trace, s6-s24; s <= 10 also brute force)

    python tests/golden/make_golden.py [--full]

--full recomputes the full-size entries (~15 min on 8 cores for the s24
triangle); without it they are carried over from the existing file.
"""
import csv
import gzip
import io
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import capf_import  # noqa: E402,F401
from capf_amd.graph import ScanGraph  # noqa: E402
from capf_amd.planner import run  # noqa: E402
from oracle import cmodel  # noqa: E402
from oracle.create_parser import parse_create  # noqa: E402
from oracle.table_np import OracleSession  # noqa: E402

LDBC = "/root/reference/morpheus-examples/src/main/resources/ldbc/csv"


def ldbc_sample():
    with gzip.open(os.path.join(LDBC, "person_0_0.csv.gz"), "rt") as f:
        persons = [int(r["id"]) for r in csv.DictReader(f, delimiter="|")]
    with gzip.open(os.path.join(LDBC, "person_knows_person_0_0.csv.gz"), "rt") as f:
        rd = csv.reader(f, delimiter="|")
        next(rd)
        knows = [[int(r[0]), int(r[1])] for r in rd]
    return {"source": "morpheus-examples/src/main/resources/ldbc/csv/person_{0_0,knows_person_0_0}.csv.gz",
            "persons": persons, "knows": knows}


def _json_value(v):
    """JSON form of the element values (CypherNode / CypherRelationship)."""
    from capf_amd.planner import CypherNode, CypherRelationship
    if isinstance(v, CypherNode):
        return {"node": v.id, "labels": sorted(v.labels), "properties": dict(v.properties)}
    if isinstance(v, CypherRelationship):
        return {"relationship": v.id, "source": v.source, "target": v.target, "type": v.rel_type,
                "properties": dict(v.properties)}
    raise TypeError(type(v).__name__)


def main():
    from reference_cases import CASES
    out = []
    for case in CASES:
        cid, src, create, query, expected = case[:5]
        opts = case[5] if len(case) > 5 else {}
        got = run(ScanGraph.from_data(OracleSession(), parse_create(create)), query, opts.get("params"))
        out.append({"id": cid, "source": src, "create": create.strip(), "expected": expected, "oracle": got,
                    "options": opts})
    with open(os.path.join(HERE, "reference_cases.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True, default=_json_value)

    if os.path.isdir(LDBC):
        with open(os.path.join(HERE, "ldbc_sample.json"), "w") as f:
            json.dump(ldbc_sample(), f)

    counts = {"rmat": {}, "params": {"a": cmodel.A, "b": cmodel.B, "c": cmodel.C, "edge_factor": 16,
                                      "seed": "0x5EED0000 + scale"}}
    path = os.path.join(HERE, "rmat_counts.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    full = "--full" in sys.argv
    if full or "full" not in old:
        counts["full"] = {str(sc): cmodel.stream_counts(sc) for sc in (20, 22, 24)}
    else:
        counts["full"] = old["full"]
    tri = dict(old.get("triangle", {})) if not full else {}
    for scale in range(6, 25, 2):
        if str(scale) in tri or (scale > 20 and not full):
            continue
        s, d = cmodel.rmat(scale)
        n = 1 << scale
        t = cmodel.count_triangle_trace(s, d, n)
        if scale <= 10:
            assert t == cmodel.count_triangle_brute(s, d, n)
        if scale <= 16:
            assert t == cmodel.count_triangle_formula(s, d, n)
        tri[str(scale)] = t
    counts["triangle"] = tri
    for scale in range(6, 17, 2):
        s, d = cmodel.rmat(scale)
        n = 1 << scale
        person = cmodel.labels(n, cmodel.rmat_seed(scale))
        counts["rmat"][str(scale)] = {
            "two_hop": int(cmodel.count_2hop(s, d, n)),
            "one_hop_person": int(cmodel.count_1hop(s, d, n, in_a=person)),
            "self_loops": int((s == d).sum()),
        }
    from ldbc import config5_query, ldbc_graph_data
    g = ScanGraph.from_data(OracleSession(), ldbc_graph_data())
    counts["ldbc_config5"] = sorted(([r["reach"], r["n"]] for r in run(g, config5_query())))
    # config 5 at its BASELINE size: LDBC-SF10-shaped KNOWS (2^16 Person nodes,
    # R-MAT edge factor 30 = 1,966,080 rels), every node a Person; the C
    # bitset BFS (oracle/rmat.c::reach_bitset), checked here against path
    # enumeration (reach_paths) on a sample of sources
    if full or "config5" not in old:
        import numpy as np
        sc5, ef5 = 16, 30
        s5, d5 = cmodel.rmat(sc5, ef5)
        n5 = 1 << sc5
        reach5 = cmodel.reach_bitset(s5, d5, n5, 3)
        sample = np.arange(0, n5, 257)
        rp, _ = cmodel.reach_paths(s5, d5, n5, sample, 3)
        assert np.array_equal(rp, reach5[sample])
        hist5 = cmodel.reach_histogram(reach5)
        with open(os.path.join(HERE, "config5_sf10.json"), "w") as f:  # compact: 14.5k [reach, n] pairs
            json.dump({"scale": sc5, "edge_factor": ef5, "upper": 3, "histogram": hist5}, f,
                      separators=(",", ":"))
        counts["config5"] = {
            "scale": sc5, "edge_factor": ef5, "nodes": n5, "rels": len(s5), "upper": 3,
            "histogram_file": "config5_sf10.json", "histogram_rows": len(hist5),
            "pairs": int(reach5.sum()),
            "sources": int((reach5 > 0).sum()),
            # Σ (a + 1)·reach[a] mod 2^63: pins reach per source, not only the histogram
            "weighted": int(((np.arange(n5, dtype=np.uint64) + 1) * reach5.astype(np.uint64)).sum()
                            % np.uint64(1 << 63)),
        }
    else:
        counts["config5"] = old["config5"]
    with open(path, "w") as f:
        json.dump(counts, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
