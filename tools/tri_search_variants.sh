#!/bin/bash
# Triangle count variants (not a test): parity subset, then s24 timing by CAPF_TRI_HASH (0 = sorted LDS copy, 1024 = LDS hash) and CAPF_TRI_ILP.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_e tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "0 2" "0 3" "0 4" "1024 2"; do
  set -- $v
  CAPF_TRI_HASH=$1 CAPF_TRI_ILP=$2 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_e_hash$1_ilp$2.txt 2>&1
done
echo done
