#!/bin/bash
# GPU test subset under its own limit: tools/gpu_tests.sh <log name> <pytest args...>
# (log under gpurun_out/; one process, per-test timeout, stops at the first failure)
name=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread -p no:cacheprovider "$@" \
  > gpurun_out/$name.log 2>&1
rc=$?
tail -15 gpurun_out/$name.log
exit $rc
