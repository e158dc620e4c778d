"""Host-overhead breakdown of one 2-hop count (not a test)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
from capf_amd.planner import plan_query, records  # noqa: E402
from capf_amd.synthetic import rmat_graph  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402
from bench import two_hop_query  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
s = GpuSession(0)
g = rmat_graph(s, scale, compact=True)
q = two_hop_query()
for _ in range(3):
    records(plan_query(g, q), ["count"])
s.sync()
tp = te = 0.0
N = 20
for _ in range(N):
    t0 = time.perf_counter()
    op = plan_query(g, q)
    t1 = time.perf_counter()
    records(op, ["count"])
    t2 = time.perf_counter()
    tp += t1 - t0
    te += t2 - t1
print(f"s{scale} plan {tp / N * 1e3:.3f} ms  execute {te / N * 1e3:.3f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    records(plan_query(g, q), ["count"])
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
