#!/bin/bash
# Triangle ILP / occupancy / LDS-copy sweep at the current kernels (not a test):
# parity subset, s24 timing by CAPF_TRI_ILP, CAPF_TRI_WPE and CAPF_TRI_SCAP.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_tests_ilp tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "4 6 1024" "4 7 768" "4 8 512" "3 8 512" "3 6 1024"; do
  set -- $v
  CAPF_TRI_ILP=$1 CAPF_TRI_WPE=$2 CAPF_TRI_SCAP=$3 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_ilp$1_wpe$2_cap$3.txt 2>&1
done
echo done
