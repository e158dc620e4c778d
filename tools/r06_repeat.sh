#!/bin/bash
# Round-6 closing evidence (not a test): the default bench line three times on
# one box (run-to-run spread of the headline), then the N-rank rehearsal.
set -e
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/repeat$i.json 2> gpurun_out/repeat$i.err
  python3 -c "import json;d=json.load(open('gpurun_out/repeat$i.json'));r=d['roofline'];print('run $i', round(d['ms_per_step'],4), round(r['frac'],4), round(r['pipeline_ms_per_query'],4), d['config'].get('ms_per_step_pipelined'))"
done
bash tools/r06_rehearse.sh
