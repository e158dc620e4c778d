#!/bin/bash
# Triangle at the lockstep-search defaults: parity, q-tile / p-block re-sweep,
# rocprof + PMC, and the bench line against the fresh PMC.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_f tests/test_gpu_parity.py tests/test_headline_sizes.py -m gpu -q -k "triangle"
for v in "24 25" "26 25" "28 25" "26 23" "26 27"; do
  set -- $v
  CAPF_TRI_QTILE=$1 CAPF_TRI_PBLOCK=$2 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_f_q$1_p$2.txt 2>&1
done
bash tools/collect_tri_profiles.sh 24 > gpurun_out/collect_tri.txt 2>&1
bash tools/pmc_tri_detail.sh 24 > gpurun_out/pmc_tri_detail.txt 2>&1
cp gpurun_out/tprof/pmc_tri_s24.json profiles/pmc_tri_s24.json
timeout -k 10 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/tri_bench.json 2> gpurun_out/tri_bench.err
echo done
