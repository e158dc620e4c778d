#!/bin/bash
# Round-3 first GPU pass at HEAD: gpu tests, smoke, default bench, profiles.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gputests.txt 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.txt 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err
bash tools/collect_profiles.sh 24 > gpurun_out/r03_collect.txt 2>&1
