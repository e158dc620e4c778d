#!/bin/bash
# Triangle at the new defaults: parity tests, the s24 bench (profiled pass gives the
# per-pass probe split), rocprof + FETCH/WRITE PMC of the count kernels, and the SQ /
# TCC detail of both passes at s24.
set -e
bash tools/gpu_tests.sh tri_tests tests/test_gpu_parity.py tests/test_headline_sizes.py -m gpu -q -k "triangle"
timeout -k 10 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/tri_bench.json 2> gpurun_out/tri_bench.err
bash tools/collect_tri_profiles.sh 24 > gpurun_out/collect_tri.txt 2>&1
bash tools/pmc_tri_detail.sh 24 > gpurun_out/pmc_tri_detail.txt 2>&1
echo done
