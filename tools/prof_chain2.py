"""Profiling driver (not a test): one warm + one measured 2-hop count at a scale.

usage: python tools/prof_chain2.py SCALE VARIANT(single|twopass) COMPACT(0|1)
Run under rocprofv3 (--kernel-trace --stats, or --pmc ...) to attribute the
partition kernels' time and traffic."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
from capf_amd.planner import run  # noqa: E402
from capf_amd.synthetic import rmat_graph  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402
from bench import two_hop_query  # noqa: E402

scale, variant, compact = int(sys.argv[1]), sys.argv[2], sys.argv[3] == "1"
os.environ["CAPF_CHAIN2"] = "partitioned"
os.environ["CAPF_C2"] = variant
s = GpuSession(0)
g = rmat_graph(s, scale, compact=compact)
q = two_hop_query()
for _ in range(2):
    c = run(g, q)[0]["count"]
s.sync()
print(f"s{scale} {variant} compact={compact} count {c}", flush=True)
