"""Host-side split of one headline query (not a test): planning (plan_query),
the count call up to its return without waiting (capf_table_count_async: DAG
analysis + launches), the wait for the device, and the whole run() path the
bench times.  Medians over N queries.

    python tools/prof_headline_host.py [scale] [n]
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
import torch  # noqa: E402

from bench import two_hop_query  # noqa: E402
from capf_amd.planner import plan_query, run  # noqa: E402
from capf_amd.synthetic import rmat_graph  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
s = GpuSession(0)
g = rmat_graph(s, scale, 16, compact=3)
q = two_hop_query()
for _ in range(5):
    run(g, q)
slot = torch.zeros(1, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
plan, call, wait, whole = [], [], [], []
for _ in range(n):
    s.sync()
    t0 = time.perf_counter()
    tbl = plan_query(g, q).table
    t1 = time.perf_counter()
    tbl.count_async(slot.data_ptr())
    t2 = time.perf_counter()
    s.sync()
    t3 = time.perf_counter()
    plan.append(t1 - t0)
    call.append(t2 - t1)
    wait.append(t3 - t2)
for _ in range(n):
    s.sync()
    t0 = time.perf_counter()
    run(g, q)
    whole.append(time.perf_counter() - t0)
us = lambda xs: statistics.median(xs) * 1e6  # noqa: E731
print(f"s{scale} medians over {n}: plan {us(plan):.1f} us, count_async call {us(call):.1f} us, "
      f"wait {us(wait):.1f} us, plan+call+wait {us([a + b + c for a, b, c in zip(plan, call, wait)]):.1f} us; "
      f"run() {us(whole):.1f} us")
