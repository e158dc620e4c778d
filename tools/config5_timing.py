"""Config 5 timing (BASELINE.json: LDBC-SNB-SF10-shaped KNOWS, *1..3
var-length + DISTINCT + GROUP BY) through the planner on one GPU.

    python tools/config5_timing.py [scale] [edge_factor] [reps]

Graph: SF10-shaped synthetic — 2^16 = 65,536 Person nodes (SF10: ≈65,645)
and R-MAT (Graph500 a/b/c) power-law KNOWS rels with edge factor 30
(1,966,080 rels; SF10: ≈1.94M directed), generated in HBM.  Query:
MATCH (a:Person)-[:KNOWS*1..3]->(b:Person) WITH DISTINCT a, b
WITH a, count(*) AS reach RETURN reach, count(*) AS n.
Reports the end-to-end time per query, the per-kernel device split (HIP
events) and, at small scales, checks the result against oracle/reach.py."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import capf_import  # noqa: E402

capf_import.load()
from ldbc import config5_query  # noqa: E402

from capf_amd.graph import ElementTable, ScanGraph  # noqa: E402
from capf_amd.planner import run  # noqa: E402
from capf_amd.synthetic import rmat_seed, thresholds  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    ef = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    s = GpuSession(0)
    m = ef << scale
    rels = s.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, m)
    nodes = s.range_nodes(0, 1 << scale, id_col="id")
    g = ScanGraph(s, [ElementTable("node", frozenset(["Person"]), nodes, {})],
                  [ElementTable("rel", frozenset(["KNOWS"]), rels, {})])
    q = config5_query()
    t0 = time.perf_counter()
    res = run(g, q)  # warm-up
    first = time.perf_counter() - t0
    s.reset_profile()
    s.set_profiling(True)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        res = run(g, q)
        ts.append(time.perf_counter() - t0)
    s.set_profiling(False)
    prof = s.profile()
    hist = sorted([r["reach"], r["n"]] for r in res)
    total_reach = sum(k * v for k, v in hist)
    print(f"config 5: {1 << scale} Person nodes, {m} KNOWS rels (R-MAT s{scale}, ef {ef}); "
          f"{sum(v for _, v in hist)} sources reach ≥1, Σ reach = {total_reach} distinct (a,b) pairs")
    print(f"  first run {first * 1e3:.1f} ms; best of {reps}: {min(ts) * 1e3:.1f} ms per query "
          f"({total_reach / min(ts) / 1e9:.2f} G distinct pairs/s)")
    dev = 0.0
    for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"]):
        ms = v["total_ms"] / reps
        dev += ms
        gbs = v["bytes"] / reps / (ms * 1e-3) / 1e9 if ms > 0 and v["bytes"] else 0.0
        print(f"  {k:14s} {ms:9.3f} ms  launches/query {v['launches'] // reps:4d}  {gbs:8.1f} GB/s (nominal bytes)")
    print(f"  profiled kernels {dev:.3f} ms per query")
    if scale <= 12:
        import numpy as np
        from oracle import reach as oreach
        src, _ = rels.column_arrays("source")
        dst, _ = rels.column_arrays("target")
        p = np.arange(1 << scale)
        assert hist == oreach.config5_histogram(src, dst, p, p), "mismatch vs oracle"
        print("  matches oracle/reach.py")
    print("  reach histogram head:", hist[:5], "tail:", hist[-3:])


if __name__ == "__main__":
    main()
