# Round profile collection on the GPU box (not a test):
#   1. rocprofv3 --kernel-trace --stats over bench.py (kernel durations)
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE) over the pipeline kernels
#   3. assemble gpurun_out/prof/pmc_s24.json (HBM bytes per query)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof
mkdir -p $OUT
SCALE=${1:-24}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 --scale $SCALE --no-cpu > $OUT/bench_traced.json 2> $OUT/trace.log
timeout -k 10 300 rocprofv3 --kernel-include-regex "c5_|c3_|chain2" --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 bench.py --steps 3 --warmup 1 --scale $SCALE --no-cpu > $OUT/bench_fetch.json 2> $OUT/fetch.log
timeout -k 10 300 rocprofv3 --kernel-include-regex "c5_|c3_|chain2" --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- python3 bench.py --steps 3 --warmup 1 --scale $SCALE --no-cpu > $OUT/bench_write.json 2> $OUT/write.log
python3 tools/make_pmc_json.py $OUT $SCALE
echo done
