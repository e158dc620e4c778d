#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 600 python -u -m pytest tests/test_headline_sizes.py -k "two_hop" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_p3dot_tests.txt 2>&1
echo "tests2"; $T 600 python -u -m pytest tests/test_gpu_parity.py -k "two_hop or chain or count" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_p3dot_tests2.txt 2>&1
for v in 1 0 1 0; do echo "bench $v"; CAPF_P3_DOT=$v $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_p3dot.jsonl 2>> gpurun_out/r03_p3dot.err; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
echo "trace"; $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt13 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/kt13.json 2> gpurun_out/kt13.err
echo done
