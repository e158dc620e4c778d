#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dense_join.py tests/test_var_length_reach.py tests/test_ldbc_config5.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_filt_tests.txt 2>&1
echo "var2"; $T 300 python3 bench.py --query var2_rows --steps 5 --warmup 2 > gpurun_out/r03_var2_filt.json 2> gpurun_out/r03_var2_filt.err
echo "rows"; $T 300 python3 bench.py --query one_hop_rows --scale 22 --steps 10 --warmup 3 > gpurun_out/r03_rows_filt.json 2> gpurun_out/r03_rows_filt.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
echo "trace var2"; $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kv3 -o kt --output-format csv -- python3 bench.py --query var2_rows --steps 3 --warmup 1 > gpurun_out/kv3.json 2> gpurun_out/kv3.err
echo done
