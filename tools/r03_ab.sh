#!/bin/bash
# A/B of pipeline variants at s24 (bench.py --no-cpu), then rocprof of the chosen one.
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "p3 variant tests"; $T 600 python -u -m pytest tests/test_headline_sizes.py -k "p3_variant or async_queue" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_ab_tests.txt 2>&1
for v in 0 1 0 1; do
  echo "bench rot=$v"; CAPF_P3_ROT=$v $T 300 python -u bench.py --no-cpu --steps 20 --warmup 5 >> gpurun_out/r03_ab_rot.jsonl 2>> gpurun_out/r03_ab_rot.err
done

echo "host split"; $T 300 python -u tools/prof_host2.py 24 > gpurun_out/r03_prof_host2.txt 2>&1
echo done2
