#!/bin/bash
# LDS-hash triangle kernels: parity, timing by table capacity / ILP; per-rank SPI
# timing at G = 8; config-5 profiles + bench line.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh tri_hash_tests tests/test_gpu_parity.py -m gpu -q -k "triangle"
for v in "0 4 1" "512 4 1" "1024 4 1" "1024 2 1" "1024 4 0"; do
  set -- $v
  CAPF_TRI_HASH=$1 CAPF_TRI_ILP=$2 CAPF_TRI_ROWS=$3 timeout -k 10 240 python -u tools/triangle_timing.py 24 > gpurun_out/tri_hash$1_ilp$2_rows$3.txt 2>&1
done
timeout -k 10 300 python -u tools/shard_spi_timing.py 24 8 > gpurun_out/shard_g8_s24.txt 2>&1
bash tools/collect_reach_profiles.sh > gpurun_out/collect_reach.txt 2>&1
cp gpurun_out/rprof/pmc_reach_s16.json profiles/pmc_reach_s16.json
timeout -k 10 300 python -u bench.py --query reach --steps 5 --warmup 2 > gpurun_out/reach_bench.json 2> gpurun_out/reach_bench.err
echo done
