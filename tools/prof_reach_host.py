"""Host side of the config-5 step (not a test): plan_query alone, plan →
device result (the histogram table's size), records() of the histogram, and a
cProfile of whole steps by own time."""
import cProfile
import os
import pstats
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
from bench import reach_query  # noqa: E402
from capf_amd.graph import ElementTable, ScanGraph  # noqa: E402
from capf_amd.planner import plan_query, records, run  # noqa: E402
from capf_amd.synthetic import rmat_seed, thresholds  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402

s = GpuSession(0)
scale, ef = 16, 30
rels = s.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, ef << scale)
nodes = s.range_nodes(0, 1 << scale, id_col="id")
g = ScanGraph(s, [ElementTable("node", frozenset(["Person"]), nodes, {})],
              [ElementTable("rel", frozenset(["KNOWS"]), rels, {})])
q = reach_query()
names = [a for a, _ in q.stages[-1].items]
for _ in range(3):
    run(g, q)
s.sync()
tp, te, tr, tt = [], [], [], []
for _ in range(20):
    t0 = time.perf_counter()
    op = plan_query(g, q)
    t1 = time.perf_counter()
    op.table.size
    t2 = time.perf_counter()
    records(op, names)
    t3 = time.perf_counter()
    tp.append(t1 - t0)
    te.append(t2 - t1)
    tr.append(t3 - t2)
    t0 = time.perf_counter()
    run(g, q)
    tt.append(time.perf_counter() - t0)
med = lambda x: statistics.median(x) * 1e3  # noqa: E731
print(f"plan {med(tp):.3f} ms, plan->size (device + fused host work) {med(te):.3f} ms, "
      f"records {med(tr):.3f} ms, whole run {med(tt):.3f} ms", flush=True)
s.reset_profile()
s.set_profiling(True)
run(g, q)
s.sync()
s.set_profiling(False)
print({k: round(v["total_ms"], 3) for k, v in s.profile().items() if v["total_ms"] > 0}, flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    run(g, q)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
