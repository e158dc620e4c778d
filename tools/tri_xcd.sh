#!/bin/bash
# Triangle XCD-grouped work cursors (not a test): parity subset, then s24 timing
# by CAPF_TRI_XCD and the grab sizes.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_xcd tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "0 4 4" "1 4 4" "1 2 2" "1 8 4" "1 1 1"; do
  set -- $v
  CAPF_TRI_XCD=$1 CAPF_TRI_GRAB_A=$2 CAPF_TRI_GRAB_B=$3 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_xcd$1_$2_$3.txt 2>&1
done
echo done
