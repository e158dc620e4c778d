"""Planner cost of the s24 2-hop count (not a test): plan_query alone, N times,
wall time per plan and a cProfile by own time (N large enough for the
3-decimal pstats columns to resolve microsecond costs)."""
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

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 16
N = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
s = GpuSession(0)
g = rmat_graph(s, scale, compact=3)
q = two_hop_query()
records(plan_query(g, q), ["count"])
s.sync()
ops = []
t0 = time.perf_counter()
for _ in range(N):
    ops.append(plan_query(g, q))
el = time.perf_counter() - t0
print(f"s{scale}: plan_query {el / N * 1e6:.1f} us per plan ({N} plans)", flush=True)
del ops
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    plan_query(g, q)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(35)
# records() of a materialised count (the scalar delivery after the device work)
import statistics  # noqa: E402
ts = []
for _ in range(200):
    op = plan_query(g, q)
    op.table.size  # runs the count
    t0 = time.perf_counter()
    records(op, ["count"])
    ts.append(time.perf_counter() - t0)
print(f"records() after the count: median {statistics.median(ts) * 1e6:.1f} us", flush=True)
