#!/bin/bash
# Bench lines of a round (not a test): headline (default run + rocprof/PMC), config 2, triangle with its CPU baseline.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
bash tools/collect_profiles.sh 24 > gpurun_out/collect_h.txt 2>&1
bash tools/collect_c2_pmc.sh > gpurun_out/collect_c2.txt 2>&1
cp gpurun_out/prof/pmc_s24.json profiles/pmc_s24.json
cp gpurun_out/prof_c2/pmc_c2_s22.json profiles/pmc_c2_s22.json
timeout -k 10 300 python -u bench.py --query one_hop_person --scale 22 --steps 10 --warmup 3 > gpurun_out/c2_bench.json 2> gpurun_out/c2_bench.err
timeout -k 10 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/tri_bench.json 2> gpurun_out/tri_bench.err
echo done
