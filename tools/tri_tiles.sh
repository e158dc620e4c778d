#!/bin/bash
# Triangle tile re-sweep at the current kernels (not a test): s24 timing by
# CAPF_TRI_QTILE (pass-A tile, log2 words) and CAPF_TRI_PBLOCK (pass-B p-block).
set -e
cd $GRAFT_REPO_ROOT
for v in "26 25" "25 25" "27 25" "26 24" "26 26"; do
  set -- $v
  CAPF_TRI_QTILE=$1 CAPF_TRI_PBLOCK=$2 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_u_q$1_p$2.txt 2>&1
done
echo done
