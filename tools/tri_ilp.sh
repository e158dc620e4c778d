#!/bin/bash
# Triangle ILP / occupancy sweep at the current kernels (not a test): parity subset,
# s24 timing by CAPF_TRI_ILP and CAPF_TRI_WPE.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_ilp tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "3 8" "4 8"; do
  set -- $v
  CAPF_TRI_ILP=$1 CAPF_TRI_WPE=$2 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_v_ilp$1_wpe$2.txt 2>&1
done
echo done
