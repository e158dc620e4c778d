#!/bin/bash
# Triangle: ids-only LDS copies + 5 waves/SIMD (not a test): parity subset, then
# s24 timing at the defaults, with one cursor for pass A, and ILP 2.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_ids tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "3 1" "3 0" "2 1"; do
  set -- $v
  CAPF_TRI_ILP=$1 CAPF_TRI_XCD_A=$2 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_ids_ilp$1_x$2.txt 2>&1
done
echo done
