"""One line per bench JSON (not a test): file, median plan->scalar ms, pipelined
ms, per-kernel ms."""
import json
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        j = json.loads(f.read().strip().splitlines()[-1])
    r = j["roofline"]
    per = {k: round(v, 4) for k, v in r.get("kernel_ms_per_query", {}).items()}
    print(path, round(j["ms_per_step"], 4), round(j["config"].get("ms_per_step_pipelined") or 0, 4), per, flush=True)
