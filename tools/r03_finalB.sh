#!/bin/bash
# Round-3 closing pass, part B: config-2 PMC + bench, triangle profiles + bench,
# rows legs, var2 rows, reach, G=8 shard timing.
set -e
mkdir -p gpurun_out/final
F=gpurun_out/final
T="timeout -k 10"
echo "c2 pmc"; bash tools/collect_c2_pmc.sh > $F/collect_c2.txt 2>&1
echo "c2 bench"; $T 300 python -u bench.py --query one_hop_person --scale 22 --steps 20 --warmup 5 --no-cpu > $F/bench_c2.json 2> $F/bench_c2.err
echo "tri profiles"; bash tools/collect_tri_profiles.sh 24 > $F/collect_tri.txt 2>&1
echo "tri bench"; $T 300 python -u bench.py --query triangle --steps 3 --warmup 1 --no-cpu > $F/bench_tri.json 2> $F/bench_tri.err
echo "rows dense"; $T 300 python -u bench.py --query one_hop_rows --scale 22 --steps 10 --warmup 3 > $F/bench_rows_dense.json 2> $F/bench_rows_dense.err
echo "rows sparse"; $T 300 python -u bench.py --query one_hop_rows --scale 22 --steps 10 --warmup 3 --id-stride 1000003 > $F/bench_rows_sparse.json 2> $F/bench_rows_sparse.err
echo "var2 rows"; $T 300 python -u bench.py --query var2_rows --steps 5 --warmup 2 > $F/bench_var2.json 2> $F/bench_var2.err
echo "reach"; $T 300 python -u bench.py --query reach --steps 5 --warmup 2 > $F/bench_reach.json 2> $F/bench_reach.err
echo "shard g8"; $T 300 python -u tools/shard_timing.py 24 8 > $F/shard_g8_s24.txt 2>&1
echo done
