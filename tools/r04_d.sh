#!/bin/bash
# Triangle count kernels: interleaved (lockstep) binary search vs LDS hash, ILP 2 / 4.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_d tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "0 4" "0 2" "1024 4" "1024 2"; do
  set -- $v
  CAPF_TRI_HASH=$1 CAPF_TRI_ILP=$2 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_d_hash$1_ilp$2.txt 2>&1
done
echo done
