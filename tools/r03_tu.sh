#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; CAPF_C3_UNITSK=0 $T 600 python -u -m pytest tests/test_headline_sizes.py -k "two_hop_headline_split or two_hop_headline_handoff or two_hop_headline[" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_tu_tests.txt 2>&1
for u in 0 1 0 1; do echo "bench $u"; CAPF_C3_UNITSK=$u $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_tu.jsonl 2>> gpurun_out/r03_tu.err; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
echo "trace"; CAPF_C3_UNITSK=0 $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt12 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/kt12.json 2> gpurun_out/kt12.err
echo done
