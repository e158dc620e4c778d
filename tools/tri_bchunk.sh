#!/bin/bash
# Triangle pass-B work-item size (not a test): s24 timing by CAPF_TRI_BCHUNK, and
# pass-B XCD cursors once more on the same box.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_bc tests/test_gpu_parity.py -m gpu -q -k "triangle_qtiled or heavy or top_id"
for v in "1024 0" "256 0" "4096 0" "16384 0" "1024 1"; do
  set -- $v
  CAPF_TRI_BCHUNK=$1 CAPF_TRI_XCD_B=$2 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_bc$1_x$2.txt 2>&1
done
echo done
