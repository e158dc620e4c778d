# Config 5 (var-length reach, SF10-shaped) profile collection on the GPU box (not a test):
#   1. rocprofv3 --kernel-trace --stats over bench.py --query reach
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE) over the vr_* kernels
#   3. gpurun_out/rprof/pmc_reach_s16.json (HBM bytes per launch)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/rprof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --query reach --steps 5 --warmup 2 --no-cpu > $OUT/bench_traced.json 2> $OUT/trace.log
timeout -k 10 300 rocprofv3 --kernel-include-regex "vr_" --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 bench.py --query reach --steps 2 --warmup 1 --no-cpu > $OUT/bench_fetch.json 2> $OUT/fetch.log
timeout -k 10 300 rocprofv3 --kernel-include-regex "vr_" --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- python3 bench.py --query reach --steps 2 --warmup 1 --no-cpu > $OUT/bench_write.json 2> $OUT/write.log
python3 tools/make_pmc_json.py $OUT 16 reach_
echo done
