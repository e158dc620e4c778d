#!/bin/bash
# Host-side profiles: config-5 step, the s24 2-hop planner, one G = 8 shard's SPI query.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/prof_reach_host.py > gpurun_out/prof_reach_host.txt 2>&1
timeout -k 10 300 python -u tools/prof_plan.py 24 3000 > gpurun_out/prof_plan_s24.txt 2>&1
SHARD_PROFILE=1 timeout -k 10 300 python -u tools/shard_spi_timing.py 24 8 0 > gpurun_out/prof_shard_g8.txt 2>&1
echo done
