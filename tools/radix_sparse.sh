#!/bin/bash
# Forced radix join on the sparse-id rows leg (MATCH (a)-->(b) RETURN a, b,
# ids v*1000003+7): bench lines + rocprofv3 kernel stats at s22 and s24, and
# the planner's choice (hashed unique index) beside them.
set -e
export TMPDIR=/tmp
o=gpurun_out/radix_sparse
mkdir -p $o
for sc in ${SCALES:-22 24}; do
CAPF_JOIN=radix timeout -k 10 300 python bench.py --query one_hop_rows --scale $sc --id-stride 1000003 --steps 5 --warmup 2 > $o/bench_radix_s$sc.json
timeout -k 10 300 python bench.py --query one_hop_rows --scale $sc --id-stride 1000003 --steps 5 --warmup 2 > $o/bench_hidx_s$sc.json
CAPF_JOIN=radix timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof$sc -o run --output-format csv -- python3 bench.py --query one_hop_rows --scale $sc --id-stride 1000003 --steps 3 --warmup 1 > $o/prof$sc.log 2>&1
find $o/prof$sc -name '*kernel_stats.csv' -exec cp {} $o/kernel_stats_radix_s$sc.csv \;
done
