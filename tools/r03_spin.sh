#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 600 python -u -m pytest tests/test_headline_sizes.py -k "two_hop" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_spin_tests.txt 2>&1
echo "tests2"; $T 600 python -u -m pytest tests/test_gpu_parity.py -k "two_hop or chain or count" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_spin_tests2.txt 2>&1
for v in 1 0 1 0; do echo "bench spin $v"; CAPF_SPIN_WAIT=$v $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_spin.jsonl 2>> gpurun_out/r03_spin.err; done
for v in 1 1; do echo "bench p3dot"; CAPF_P3_DOT=$v $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_spin_p3dot.jsonl 2>> gpurun_out/r03_spin.err; done
echo done
