#!/bin/bash
# Filter fused into the radix join's EMIT: full GPU suite, var2 rows leg (fused / join-then-filter),
# rocprof kernel trace of the fused leg.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh full_h tests/ -m gpu -q
timeout -k 10 300 python -u bench.py --query var2_rows --scale 14 --steps 5 --warmup 2 --no-cpu > gpurun_out/var2_fused.json 2> gpurun_out/var2_fused.err
CAPF_RJ_FILTER=0 timeout -k 10 300 python -u bench.py --query var2_rows --scale 14 --steps 5 --warmup 2 --no-cpu > gpurun_out/var2_unfused.json 2> gpurun_out/var2_unfused.err
mkdir -p gpurun_out/prof_var2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_var2/fused -o var2 --output-format csv -- python3 bench.py --query var2_rows --scale 14 --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_var2/bench.json 2> gpurun_out/prof_var2/trace.log
echo done
