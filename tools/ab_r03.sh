#!/bin/bash
# A/B on one box (not a test): the round-3 tree (_r03, built in place) against
# HEAD, headline bench alternated.
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  (cd _r03 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > ../gpurun_out/ab_r03_$i.json 2> ../gpurun_out/ab_r03_$i.err)
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab_r04_$i.json 2> gpurun_out/ab_r04_$i.err
done
echo done
