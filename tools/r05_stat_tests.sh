#!/bin/bash
# Round-5 GPU check (not a test): the new aggregators / UNWIND / math tests and the reference cases, then the headline bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_comm_gpu.py -k "stdev or percentiles or unwind or math or case_atan2 or comm" \
  > gpurun_out/r05_stat.log 2>&1
rc=$?
tail -5 gpurun_out/r05_stat.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r05_base_bench.json 2> gpurun_out/r05_base_bench.err
