#!/bin/bash
# Round-6 closing measurement on the GPU box (not a test): the rocprof kernel
# trace + FETCH/WRITE PMC passes of the headline (tools/collect_profiles.sh),
# then the default bench line and smoke(), each under its own time limit;
# stops at the first failure.
set -e
bash tools/collect_profiles.sh 24 > gpurun_out/closing_prof.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/closing_bench.json 2> gpurun_out/closing_bench.err
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/closing_smoke.log 2>&1
python3 -c "import json;d=json.load(open('gpurun_out/closing_bench.json'));r=d['roofline'];print(d['ms_per_step'], r['frac'], r.get('kernel_event_frac'), d['config'].get('ms_per_step_pipelined'), d['config'].get('lib'))"
cat gpurun_out/closing_smoke.log | tail -2
