#!/bin/bash
# Round-4 check: GPU test suite, 2-rank bench rehearsal through the SPI, then the
# s24 triangle with the pass-A q-tile sweep (each step under its own limit).
set -e
bash tools/gpu_tests.sh full2 tests -m gpu -q
timeout -k 10 300 python -u bench.py --gpus 2 --one-device --scale 20 --steps 5 --warmup 2 > gpurun_out/dist2.json 2> gpurun_out/dist2.err
for qt in 0 20 22 24; do
  CAPF_TRI_QTILE=$qt timeout -k 10 300 python -u bench.py --query triangle --steps 3 --warmup 1 --no-cpu > gpurun_out/tri_q$qt.json 2> gpurun_out/tri_q$qt.err
  python3 -c "import json;j=json.load(open('gpurun_out/tri_q$qt.json'));print('qtile $qt', j['ms_per_step'], j['config']['first_query_ms'], j['config']['parity'])"
done
