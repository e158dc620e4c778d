"""Ad-hoc (not a test): device time of ONE rank's share of the node-partitioned
2-hop count at world size G, run on a single GPU (rank `part` of G), to
predict the N-GPU step before an N-GPU node is available.
usage: python tools/shard_timing.py SCALE G [PART]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
import torch  # noqa: E402
from capf_amd.dist import node_partitioned_copies  # noqa: E402
from capf_amd.synthetic import rmat_seed, thresholds  # noqa: E402
from capf_amd.table import GpuSession, chain2_sharded_count_async  # noqa: E402

scale, G = int(sys.argv[1]), int(sys.argv[2])
parts = [int(sys.argv[3])] if len(sys.argv) > 3 else list(range(G))
s = GpuSession.on_torch_stream(0)
m, n = 16 << scale, 1 << scale
full = s.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, m)
tot = 0
for p in parts:
    ic, oc = node_partitioned_copies(full, n, G, p, compact=int(os.environ.get("CAPF_WIDTH", "3")))
    partial = torch.zeros(1, dtype=torch.int64, device="cuda")
    run = lambda: chain2_sharded_count_async(s, ic, oc, 0, n, G, p, partial.data_ptr())  # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        run()
        v = int(partial.item())
    el = (time.perf_counter() - t0) / 10
    s.reset_profile()
    s.set_profiling(True)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    s.set_profiling(False)
    prof = {k: round(x["total_ms"] / 5, 4) for k, x in s.profile().items()}
    # host cost of enqueueing one step (what bounds a pipelined N-GPU bench when
    # it exceeds the device time): 20 async steps without a sync in between
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(20):
        run()
    enq = (time.perf_counter() - t1) / 20
    torch.cuda.synchronize()
    dev = sum(prof.values())
    tot += v
    print(f"s{scale} G={G} part {p}: in {ic.size} out {oc.size} rows (hot {getattr(oc, 'hot_ids', [])}); "
          f"step {el*1e3:.3f} ms enqueue {enq*1e3:.3f} ms "
          f"dev {dev:.3f} ms {prof} partial {v}", flush=True)
print("sum of partials", tot)
