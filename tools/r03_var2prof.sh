#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "radix tests"; $T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dense_join.py -k "radix or join" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_rj_tests.txt 2>&1
echo "var2"; $T 300 python3 bench.py --query var2_rows --steps 3 --warmup 1 > gpurun_out/r03_var2_u4.json 2> gpurun_out/r03_var2_u4.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
echo "trace var2"; $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kv2 -o kt --output-format csv -- python3 bench.py --query var2_rows --steps 3 --warmup 1 > gpurun_out/kv2.json 2> gpurun_out/kv2.err
echo "dot grids"; for g in 512 1024; do CAPF_DOT_GRID=$g $T 300 python3 bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_dotgrid.jsonl 2>>gpurun_out/r03_dotgrid.err; done
echo done
