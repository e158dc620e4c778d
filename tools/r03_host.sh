#!/bin/bash
# host-side split of the s24 2-hop query, then the GPU test suite
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prof_host2.py 24 > gpurun_out/r03_prof_host2.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gputests.txt 2>&1
