#!/bin/bash
# Round-3 closing pass (short): triangle bench, sparse rows leg, G=8 shard timing.
set -e
mkdir -p gpurun_out/final
F=gpurun_out/final
T="timeout -k 10"
echo "tri bench"; $T 300 python -u bench.py --query triangle --steps 3 --warmup 1 --no-cpu > $F/bench_tri.json 2> $F/bench_tri.err
echo "rows sparse"; $T 300 python -u bench.py --query one_hop_rows --scale 22 --steps 10 --warmup 3 --id-stride 1000003 > $F/bench_rows_sparse.json 2> $F/bench_rows_sparse.err
echo "shard g8"; $T 300 python -u tools/shard_timing.py 24 8 > $F/shard_g8_s24.txt 2>&1
echo done
