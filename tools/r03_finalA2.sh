#!/bin/bash
# Round-3 closing pass: headline bench with the CPU baseline, rocprof trace + PMC.
set -e
mkdir -p gpurun_out/final
F=gpurun_out/final
T="timeout -k 10"
echo "bench"; $T 400 python -u bench.py --steps 30 --warmup 5 > $F/bench_s24.json 2> $F/bench_s24.err
echo "profiles"; bash tools/collect_profiles.sh 24 > $F/collect.txt 2>&1
echo done
