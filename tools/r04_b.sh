#!/bin/bash
# Triangle load/search split (CAPF_TRI_DIAG), config-5 profiles + bench line,
# per-rank SPI timing of the node-partitioned 2-hop count at G = 8.
set -e
cd $GRAFT_REPO_ROOT
for d in 0 1 2; do
  CAPF_TRI_DIAG=$d timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_diag$d.txt 2>&1
done
timeout -k 10 300 python -u tools/shard_spi_timing.py 24 8 > gpurun_out/shard_g8_s24.txt 2>&1
bash tools/collect_reach_profiles.sh > gpurun_out/collect_reach.txt 2>&1
cp gpurun_out/rprof/pmc_reach_s16.json profiles/pmc_reach_s16.json
timeout -k 10 300 python -u bench.py --query reach --steps 5 --warmup 2 > gpurun_out/reach_bench.json 2> gpurun_out/reach_bench.err
echo done
