#!/bin/bash
# Triangle work-queue grab sizes (not a test): parity subset, then s24 timing by
# CAPF_TRI_GRAB_A / CAPF_TRI_GRAB_B, and the staging-only diagnostic.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_grab tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "4 4 0" "32 8 0" "64 16 0" "128 32 0" "32 8 3"; do
  set -- $v
  CAPF_TRI_GRAB_A=$1 CAPF_TRI_GRAB_B=$2 CAPF_TRI_DIAG=$3 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_grab$1_$2_d$3.txt 2>&1
done
echo done
