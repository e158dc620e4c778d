#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 600 python -u -m pytest tests/test_headline_sizes.py tests/test_gpu_parity.py tests/test_dense_join.py -k "two_hop or handoff or radix or join" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_fuse6_tests.txt 2>&1
for i in 1 2; do echo "bench $i"; $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_fuse6_bench.jsonl 2>> gpurun_out/r03_fuse6_bench.err; done
echo "bench grid512"; CAPF_DOT_GRID=512 $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_fuse6_bench.jsonl 2>> gpurun_out/r03_fuse6_bench.err
echo "var2 rows"; $T 300 python -u bench.py --query var2_rows --steps 3 --warmup 1 > gpurun_out/r03_var2_rows_pc.json 2> gpurun_out/r03_var2_rows_pc.err
echo "var2 rows pc64"; CAPF_RJ_PCHUNK=64 $T 300 python -u bench.py --query var2_rows --steps 3 --warmup 1 > gpurun_out/r03_var2_rows_pc64.json 2> gpurun_out/r03_var2_rows_pc64.err
echo "trace"; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt8 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/kt8.json 2> gpurun_out/kt8.err
echo done
