#!/bin/bash
# Round-5 GPU check after pruning the kept-off variants (not a test): the
# headline-size fixtures, the 2-hop / sharded / triangle parity subset, then
# the headline profile (kernel trace + PMC passes + planner cost).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_headline_sizes.py tests/test_gpu_parity.py -k "headline or two_hop or chain2 or sharded or triangle or tri_" \
  > gpurun_out/r05_prune.log 2>&1
rc=$?
tail -5 gpurun_out/r05_prune.log
[ $rc -ne 0 ] && exit $rc
bash tools/r05_headline_prof.sh
