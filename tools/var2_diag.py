import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import capf_import  # noqa
from capf_amd.planner import plan_query
from capf_amd.synthetic import rmat_graph
from capf_amd.table import GpuSession
from bench import var2_rows_query
s = GpuSession(0)
g = rmat_graph(s, 12, 16, compact=True)
q = var2_rows_query()
plan_query(g, q).table.materialize(); s.sync()
s.reset_profile(); s.set_profiling(True)
t = plan_query(g, q).table
t.materialize(); s.sync()
s.set_profiling(False)
for k, v in s.profile().items():
    print(k, v)
