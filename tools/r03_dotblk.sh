#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; CAPF_DOT_BLOCK=1024 $T 600 python -u -m pytest tests/test_headline_sizes.py -k "two_hop" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_dotblk_tests.txt 2>&1
for b in 256 512 1024 256 1024; do echo "bench $b"; CAPF_DOT_BLOCK=$b $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_dotblk.jsonl 2>> gpurun_out/r03_dotblk.err; done
echo done
