#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 600 python -u -m pytest tests/test_headline_sizes.py -k "two_hop" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_fuse7_tests.txt 2>&1
echo "tests2"; $T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_fuse7_tests2.txt 2>&1
for i in 1 2; do echo "bench $i"; $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_fuse7_bench.jsonl 2>> gpurun_out/r03_fuse7_bench.err; done
echo "bench unitsk"; CAPF_C3_UNITSK=1 $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_fuse7_bench.jsonl 2>> gpurun_out/r03_fuse7_bench.err
echo "trace"; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt9 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/kt9.json 2> gpurun_out/kt9.err
echo done
