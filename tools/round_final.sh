#!/bin/bash
# Closing checks of a round (not a test): full GPU suite, smoke, the default
# bench line (headline), the config-5 line, the s24 planner profile.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh full_closing tests/ -m gpu -q
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.txt 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
timeout -k 10 300 python -u bench.py --query reach --steps 5 --warmup 2 > gpurun_out/reach_bench.json 2> gpurun_out/reach_bench.err
timeout -k 10 300 python -u tools/prof_plan.py 24 3000 > gpurun_out/prof_plan_s24.txt 2>&1
echo done
