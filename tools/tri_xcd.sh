#!/bin/bash
# Triangle XCD-grouped work cursors (not a test): parity subset, then s24 timing
# by CAPF_TRI_XCD_A / _B (grabs per XCD chunk, 0 = one cursor) and the grab sizes.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_xcd tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "64 0 2 4" "16 0 2 4" "256 0 2 4" "64 64 2 4" "64 16 2 2" "64 0 1 4"; do
  set -- $v
  CAPF_TRI_XCD_A=$1 CAPF_TRI_XCD_B=$2 CAPF_TRI_GRAB_A=$3 CAPF_TRI_GRAB_B=$4 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_w_x$1_$2_g$3_$4.txt 2>&1
done
echo done
