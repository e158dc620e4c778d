"""Host-side split of one 2-hop query at scale s (not a test): plan, enqueue of
the fused count, wait for the GPU, scalar readback; cProfile of the planner by
own time."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
import torch  # noqa: E402
from capf_amd.planner import plan_query, records  # noqa: E402
from capf_amd.synthetic import rmat_graph  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402
from bench import two_hop_query  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
s = GpuSession(0)
g = rmat_graph(s, scale, compact=3)
q = two_hop_query()
for _ in range(3):
    records(plan_query(g, q), ["count"])
s.sync()
slot = torch.zeros(1, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
N = 30
rows = []
for _ in range(N):
    s.sync()
    t0 = time.perf_counter()
    op = plan_query(g, q)
    t1 = time.perf_counter()
    op.table.count_async(slot.data_ptr())
    t2 = time.perf_counter()
    s.sync()
    t3 = time.perf_counter()
    records(op, ["count"])
    t4 = time.perf_counter()
    rows.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3))
rows.sort(key=lambda r: sum(r))
med = rows[len(rows) // 2]
print(f"s{scale} median query: plan {med[0]*1e3:.3f} ms  enqueue {med[1]*1e3:.3f}  wait {med[2]*1e3:.3f}  "
      f"records(size, memoised) {med[3]*1e3:.3f}", flush=True)
for name, fn in (("plan", lambda: plan_query(g, q)),):
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(N):
        fn()
    pr.disable()
    print(f"--- {name}: cProfile by tottime over {N} plans")
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
