"""Host-side profile of the config-5 query (not a test)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import config5_timing as c5  # noqa: E402

s = c5.GpuSession(0)
scale, ef = 16, 30
rels = s.rmat_rels(scale, c5.rmat_seed(scale), c5.thresholds(), 0, ef << scale)
nodes = s.range_nodes(0, 1 << scale, id_col="id")
g = c5.ScanGraph(s, [c5.ElementTable("node", frozenset(["Person"]), nodes, {})],
                 [c5.ElementTable("rel", frozenset(["KNOWS"]), rels, {})])
q = c5.config5_query()
c5.run(g, q)
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    c5.run(g, q)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
