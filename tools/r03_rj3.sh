#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 900 python -u -m pytest tests/test_gpu_parity.py -k "filter or reference or join" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_rj3_tests.txt 2>&1
echo "var2"; $T 300 python3 bench.py --query var2_rows --steps 5 --warmup 2 > gpurun_out/r03_var2_rj3.json 2> gpurun_out/r03_var2_rj3.err
echo done
