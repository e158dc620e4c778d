"""Determinism check of the fused 2-hop count (ad-hoc)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa
from capf_amd.table import GpuSession
from capf_amd.synthetic import rmat_graph
from capf_amd.planner import run
from bench import two_hop_query
scale = int(sys.argv[1]); mode = sys.argv[2]
os.environ["CAPF_CHAIN2"] = mode
s = GpuSession(0)
g = rmat_graph(s, scale)
q = two_hop_query()
out = []
for i in range(4):
    t = time.perf_counter()
    out.append(run(g, q)[0]["count"])
    out.append(round((time.perf_counter() - t) * 1e3, 2))
print(f"s{scale} {mode} alloc={os.environ.get('CAPF_ALLOC','pool')} poison={os.environ.get('CAPF_POISON','0')}", out, flush=True)
