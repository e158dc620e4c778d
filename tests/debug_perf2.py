"""Ad-hoc: compare partition variants × id encodings at a scale (not a test)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capf_import  # noqa
from capf_amd.table import GpuSession
from capf_amd.synthetic import rmat_graph
from capf_amd.planner import run
from bench import two_hop_query
scale = int(sys.argv[1])
variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["single", "twopass"]
s = GpuSession(0)
q = two_hop_query()
os.environ["CAPF_CHAIN2"] = "partitioned"
for compact in (False, True):
    g = rmat_graph(s, scale, compact=compact)
    for variant in variants:
        os.environ["CAPF_C2"] = variant
        c = run(g, q)[0]["count"]
        s.sync(); s.reset_profile(); s.set_profiling(True)
        t = time.perf_counter()
        for _ in range(5):
            c2 = run(g, q)[0]["count"]
        s.sync()
        el = (time.perf_counter() - t) / 5
        s.set_profiling(False)
        prof = {k: round(v["total_ms"] / v["launches"], 3) for k, v in s.profile().items()}
        enc = "for32" if compact else "int64"
        print(f"s{scale} {enc} {variant:8s} count {c} {c2} step {el*1e3:.3f} ms  kernels {prof}",
              flush=True)
    del g
