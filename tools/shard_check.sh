#!/bin/bash
# Multi-GPU SPI path (not a test): the 2-/3-rank GPU tests, then the per-rank
# timing at G = 8 (all parts) and a cProfile of part 0.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh dist_gpu tests/test_dist_gpu.py -m gpu -q
timeout -k 10 300 python -u tools/shard_spi_timing.py 24 8 > gpurun_out/shard_g8_s24.txt 2>&1
SHARD_PROFILE=1 timeout -k 10 300 python -u tools/shard_spi_timing.py 24 8 0 > gpurun_out/prof_shard_g8.txt 2>&1
echo done
