"""Ad-hoc: sweep the P3 shape (not a test)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa
from capf_amd.table import GpuSession
from capf_amd.synthetic import rmat_graph
from capf_amd.planner import run
from bench import two_hop_query
scale = int(sys.argv[1])
s = GpuSession(0)
q = two_hop_query()
g = rmat_graph(s, scale, compact=True)
for shape in sys.argv[2].split(";"):
    os.environ["CAPF_P3"] = shape
    c = run(g, q)[0]["count"]
    s.sync(); s.reset_profile(); s.set_profiling(True)
    for _ in range(5):
        c2 = run(g, q)[0]["count"]
    s.sync(); s.set_profiling(False)
    prof = {k: round(v["total_ms"] / v["launches"], 3) for k, v in s.profile().items()}
    print(f"s{scale} P3 {shape} count {c} {c2} kernels {prof}", flush=True)
