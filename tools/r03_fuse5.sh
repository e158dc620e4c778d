#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 900 python -u -m pytest tests/test_headline_sizes.py tests/test_gpu_parity.py tests/test_dense_join.py -k "two_hop or triangle or join or radix or reference" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_fuse5_tests.txt 2>&1
for i in 1 2; do echo "bench $i"; $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_fuse5_bench.jsonl 2>> gpurun_out/r03_fuse5_bench.err; done
echo "var2 rows"; $T 300 python -u bench.py --query var2_rows --steps 3 --warmup 1 > gpurun_out/r03_var2_rows_runs.json 2> gpurun_out/r03_var2_rows_runs.err
for pb in 24 22 26; do echo "tri pblock $pb"; CAPF_TRI_PBLOCK=$pb $T 300 python -u bench.py --query triangle --steps 3 --warmup 1 >> gpurun_out/r03_tri_pb.jsonl 2>> gpurun_out/r03_tri_pb.err; done
echo "trace"; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt7 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/kt7.json 2> gpurun_out/kt7.err
echo done
