#!/bin/bash
# Triangle profiles of a round (not a test): triangle parity subset first, then
# rocprof + FETCH/WRITE PMC + the SQ/TCC detail at s24, and the bench line
# against the fresh PMC.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_final tests/test_gpu_parity.py tests/test_headline_sizes.py -m gpu -q -k "triangle"
bash tools/collect_tri_profiles.sh 24 > gpurun_out/collect_tri.txt 2>&1
bash tools/pmc_tri_detail.sh 24 > gpurun_out/pmc_tri_detail.txt 2>&1
cp gpurun_out/tprof/pmc_tri_s24.json profiles/pmc_tri_s24.json
timeout -k 10 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/tri_bench.json 2> gpurun_out/tri_bench.err
echo done
