"""Ad-hoc (not a test): per-kernel device time of the fused 2-hop count under
environment variants.  usage: python tools/prof_variants.py SCALE 'ENV=..;ENV2=..' ['...']
An empty spec '' is the default configuration."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa: E402,F401
from bench import two_hop_query  # noqa: E402
from capf_amd.planner import run  # noqa: E402
from capf_amd.synthetic import rmat_graph  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402

scale = int(sys.argv[1])
s = GpuSession(0)
_w = os.environ.get("CAPF_WIDTH", "3")  # id storage: 3 = FOR24, 4 = FOR32, 8 = int64
g = rmat_graph(s, scale, compact={"3": 3, "4": True, "8": False}[_w])
q = two_hop_query()
base = dict(os.environ)
for spec in sys.argv[2:]:
    os.environ.clear()
    os.environ.update(base)
    for kv in filter(None, spec.split(";")):
        k, v = kv.split("=")
        os.environ[k] = v
    c = run(g, q)[0]["count"]
    run(g, q)
    s.sync()
    t = time.perf_counter()
    for _ in range(5):
        run(g, q)
    s.sync()
    el = (time.perf_counter() - t) / 5
    s.reset_profile()
    s.set_profiling(True)
    for _ in range(5):
        c2 = run(g, q)[0]["count"]
    s.sync()
    s.set_profiling(False)
    prof = {k: round(v["total_ms"] / v["launches"], 4) for k, v in s.profile().items()}
    tot = sum(v["total_ms"] for v in s.profile().values()) / 5
    print(f"s{scale} [{spec}] count {c} {c2} step {el*1e3:.3f} ms dev {tot:.3f} ms {prof}", flush=True)
