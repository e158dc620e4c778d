#!/bin/bash
# Round-3 closing pass, part A: full gpu suite, smoke, headline bench (CPU baseline),
# rocprof kernel trace + PMC of the s24 pipeline.
set -e
mkdir -p gpurun_out/final
F=gpurun_out/final
T="timeout -k 10"
echo "suite"; $T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gputests.txt 2>&1
echo "smoke"; $T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1
echo "bench"; $T 400 python -u bench.py --steps 30 --warmup 5 > $F/bench_s24.json 2> $F/bench_s24.err
echo "profiles"; bash tools/collect_profiles.sh 24 > $F/collect.txt 2>&1
echo done
