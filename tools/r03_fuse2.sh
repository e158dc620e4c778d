#!/bin/bash
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "tests"; $T 900 python -u -m pytest tests/test_headline_sizes.py -k "two_hop" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_fuse4_tests.txt 2>&1
for i in 1 2; do echo "bench $i"; $T 300 python -u bench.py --no-cpu --steps 30 --warmup 5 >> gpurun_out/r03_fuse4_bench.jsonl 2>> gpurun_out/r03_fuse4_bench.err; done
echo "trace"; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt6 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/kt6.json 2> gpurun_out/kt6.err
echo "plan prof"; $T 300 python -u tools/prof_plan.py 16 3000 > gpurun_out/r03_prof_plan3.txt 2>&1
echo "var2 rows"; $T 300 python -u bench.py --query var2_rows --steps 3 --warmup 1 > gpurun_out/r03_var2_rows.json 2> gpurun_out/r03_var2_rows.err
echo done
