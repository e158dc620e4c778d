#!/bin/bash
# Fused post-P1 pipeline (no memsets / zero / overflow / D2H launches) + two-pass triangle:
# tests, bench A/B, kernel trace.
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 900 python -u -m pytest tests/test_headline_sizes.py tests/test_gpu_parity.py tests/test_dist_gpu.py -k "two_hop or chain2 or triangle or dist or hist or partitioned or loops" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_fuse_tests.txt 2>&1
for i in 1 2; do echo "bench $i"; $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_fuse_bench.jsonl 2>> gpurun_out/r03_fuse_bench.err; done
echo "tri two-pass"; $T 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/r03_tri_2p.json 2> gpurun_out/r03_tri_2p.err
echo "tri one-pass"; CAPF_TRI_TWOPASS=0 $T 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/r03_tri_1p.json 2> gpurun_out/r03_tri_1p.err
echo "trace"; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt3 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/kt3.json 2> gpurun_out/kt3.err
echo done
