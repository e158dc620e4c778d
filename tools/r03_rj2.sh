#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dense_join.py -k "radix or join or reference" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_rj2_tests.txt 2>&1
echo "var2"; $T 300 python3 bench.py --query var2_rows --steps 5 --warmup 2 > gpurun_out/r03_var2_rj2.json 2> gpurun_out/r03_var2_rj2.err
echo "var2 s16"; $T 300 python3 bench.py --query var2_rows --scale 16 --steps 3 --warmup 1 > gpurun_out/r03_var2_rj2_s16.json 2> gpurun_out/r03_var2_rj2_s16.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
echo "trace var2"; $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kv4 -o kt --output-format csv -- python3 bench.py --query var2_rows --steps 3 --warmup 1 > gpurun_out/kv4.json 2> gpurun_out/kv4.err
echo done
