"""Ad-hoc (not a test): ONE rank's share of the node-partitioned 2-hop count at
world size G through the Table SPI — planner.run on the rank's DistTable graph
(dist_table.dist_node_partitioned_graph), DistTable.group(∅, count(*))
dispatching capf_chain2_sharded_count, the int64 all-reduce (an RCCL group of
one rank here: the 8-GPU exchange cannot run on a 1-GPU box) and the host read —
timed per query (plan call → scalar: host + device), rank `part` of G run on
this GPU one after the other.  Also the device time of the rank's kernels.
usage: python tools/shard_spi_timing.py SCALE G [PART ...]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from capf_amd.dist_table import DistSession, GpuExchange, dist_node_partitioned_graph  # noqa: E402
from capf_amd.graph import ElementTable, ScanGraph  # noqa: E402
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run  # noqa: E402
from capf_amd.expr import CountStar  # noqa: E402
from capf_amd.synthetic import rmat_seed, thresholds  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402


class SoloExchange(GpuExchange):
    """Rank `rank` of `world` on this GPU: row routing as on the real ranks,
    no collectives on host values (the graph build asks none for this layout)."""

    def __init__(self, s, world, rank):
        self.s, self.group, self.world, self.rank = s, None, world, rank
        self.staged, self.dev = False, torch.device("cuda", 0)

    def all_sum(self, v):
        return int(v)


scale, G = int(sys.argv[1]), int(sys.argv[2])
parts = [int(x) for x in sys.argv[3:]] or list(range(G))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29577")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
s = GpuSession.on_torch_stream(0)
m, n = 16 << scale, 1 << scale
q = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
          [Stage([("count", CountStar())])])
tot, worst = 0, 0.0
for p in parts:
    full = s.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, m)
    nodes = s.range_nodes(0, n, id_col="id")
    ds = DistSession(s, SoloExchange(s, G, p))
    g = dist_node_partitioned_graph(ds, ScanGraph(s, [ElementTable("node", frozenset(), nodes, {})],
                                                  [ElementTable("rel", frozenset(["E"]), full, {})]),
                                    compact=int(os.environ.get("CAPF_WIDTH", "3")))
    del full, nodes
    for _ in range(5):
        v = run(g, q)[0]["count"]
    times = []
    for _ in range(30):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        v = run(g, q)[0]["count"]
        times.append(time.perf_counter() - t0)
    plan = []
    from capf_amd.planner import plan_query
    for _ in range(30):
        t0 = time.perf_counter()
        plan_query(g, q)
        plan.append(time.perf_counter() - t0)
    s.reset_profile()
    s.set_profiling(True)
    for _ in range(5):
        run(g, q)
    torch.cuda.synchronize()
    s.set_profiling(False)
    prof = {k: round(x["total_ms"] / 5, 4) for k, x in s.profile().items() if x["total_ms"] > 0}
    med = statistics.median(times) * 1e3
    worst = max(worst, med)
    tot += v
    print(f"s{scale} G={G} part {p}: plan->scalar median {med:.3f} ms (min {min(times)*1e3:.3f}), "
          f"planning alone {statistics.median(plan)*1e3:.3f} ms, device {sum(prof.values()):.3f} ms {prof}, "
          f"partial {v}", flush=True)
    if os.environ.get("SHARD_PROFILE") == "1":  # where the host time of a query goes
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(200):
            run(g, q)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    del g, ds
print(f"sum of partials {tot}; max over parts of the median plan->scalar {worst:.3f} ms")
dist.destroy_process_group()
