#!/bin/bash
# Triangle batch-owner search (not a test): parity subset, then s24 timing with
# CAPF_TRI_GALLOP 1 / 0 and the staging-only diagnostic (CAPF_TRI_DIAG=3).
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_g tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "1 0" "0 0" "1 3"; do
  set -- $v
  CAPF_TRI_GALLOP=$1 CAPF_TRI_DIAG=$2 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_g$1_d$2.txt 2>&1
done
echo done
