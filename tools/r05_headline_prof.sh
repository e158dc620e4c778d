#!/bin/bash
# Headline profile of a round (not a test): kernel trace + stats, FETCH/WRITE PMC passes, planner cost.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/collect_profiles.sh 24 > gpurun_out/collect_h.txt 2>&1
timeout -k 10 200 python3 tools/prof_plan.py 24 2000 > gpurun_out/prof_plan_s24.txt 2>&1
echo done
