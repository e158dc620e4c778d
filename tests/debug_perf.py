"""Ad-hoc: compare chain2 modes at a scale (profiled kernel times)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa
from capf_amd.table import GpuSession
from capf_amd.synthetic import rmat_graph
from capf_amd.planner import run
from bench import two_hop_query

scale = int(sys.argv[1])
s = GpuSession(0)
g = rmat_graph(s, scale)
q = two_hop_query()
for mode in ("atomic", "partitioned", "atomic", "partitioned"):
    os.environ["CAPF_CHAIN2"] = mode
    c = run(g, q)[0]["count"]
    s.sync(); s.reset_profile(); s.set_profiling(True)
    t = time.perf_counter()
    for _ in range(5):
        c2 = run(g, q)[0]["count"]
    s.sync()
    el = (time.perf_counter() - t) / 5
    s.set_profiling(False)
    prof = {k: round(v["total_ms"] / v["launches"], 3) for k, v in s.profile().items()}
    print(f"s{scale} {mode:12s} count {c} {c2} step {el*1e3:.3f} ms  kernels {prof}", flush=True)
