"""Ad-hoc (not a test): the fused triangle count (config 4 shape) on R-MAT at
the given scales — wall time through the planner and the per-kernel split.
usage: python tools/triangle_timing.py SCALE [SCALE ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
from bench import triangle_query  # noqa: E402
from capf_amd.planner import run  # noqa: E402
from capf_amd.synthetic import rmat_graph  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402

s = GpuSession(0)
q = triangle_query()
for scale in map(int, sys.argv[1:]):
    g = rmat_graph(s, scale, compact=True)
    c = run(g, q)[0]["count"]
    s.sync()
    t = time.perf_counter()
    c2 = run(g, q)[0]["count"]
    el = time.perf_counter() - t
    s.reset_profile()
    s.set_profiling(True)
    run(g, q)
    s.sync()
    s.set_profiling(False)
    prof = {k: round(v["total_ms"], 2) if v["total_ms"] > 0 else v["bytes"] for k, v in s.profile().items()}
    print(f"s{scale} triangle count {c} {c2} plan {s.last_plan()} {el*1e3:.1f} ms {prof}", flush=True)
    del g
