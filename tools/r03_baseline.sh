#!/bin/bash
# Round-3 baseline: headline bench (no CPU leg) + host-side profile of one 2-hop query at s24.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r03_bench_base.json 2> gpurun_out/r03_bench_base.err
timeout -k 10 300 python -u tools/prof_host.py 24 > gpurun_out/r03_prof_host.txt 2>&1
