#!/bin/bash
# round-6 GPU step: the -m gpu suite, then the config-5 host split (tools/prof_reach_host.py)
bash tools/gpu_tests.sh r06_suite2 tests -m gpu
rc=$?
echo "suite rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python tools/prof_reach_host.py > gpurun_out/r06_reach_host.txt 2>&1 || exit $?
head -3 gpurun_out/r06_reach_host.txt
