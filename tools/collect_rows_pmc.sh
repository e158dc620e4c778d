#!/bin/bash
# Sparse-id rows leg PMC traffic (not a test): FETCH_SIZE / WRITE_SIZE passes
# over the hashed-index probes of bench.py --query one_hop_rows --id-stride
# 1000003 → gpurun_out/prof_rows/pmc_rows_sparse_s22.json
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_rows
mkdir -p $OUT
ARGS="--query one_hop_rows --scale 22 --id-stride 1000003 --steps 5 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-include-regex "hidx_probe" --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/fetch.log
timeout -k 10 300 rocprofv3 --kernel-include-regex "hidx_probe" --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- python3 bench.py $ARGS > $OUT/bench_write.json 2> $OUT/write.log
python3 tools/make_pmc_json.py $OUT 22 rows_sparse_
echo done
