#!/bin/bash
# Round-3 closing pass (short): config-2 PMC + bench, var2 rows leg.
set -e
mkdir -p gpurun_out/final
F=gpurun_out/final
T="timeout -k 10"
echo "c2 pmc"; bash tools/collect_c2_pmc.sh > $F/collect_c2.txt 2>&1
echo "c2 bench"; $T 300 python -u bench.py --query one_hop_person --scale 22 --steps 20 --warmup 5 --no-cpu > $F/bench_c2.json 2> $F/bench_c2.err
echo "var2 rows"; $T 300 python -u bench.py --query var2_rows --steps 5 --warmup 2 > $F/bench_var2.json 2> $F/bench_var2.err
echo done
