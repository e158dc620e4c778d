# Triangle (config 4) profile collection on the GPU box (not a test):
#   1. rocprofv3 --kernel-trace --stats over bench.py --query triangle
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE) over the triangle kernels
#   3. gpurun_out/tprof/pmc_tri_s<scale>.json (HBM bytes per launch)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tprof
mkdir -p $OUT
SCALE=${1:-24}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --query triangle --steps 3 --warmup 1 --scale $SCALE --no-cpu > $OUT/bench_traced.json 2> $OUT/trace.log
timeout -k 10 300 rocprofv3 --kernel-include-regex "tri_" --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 bench.py --query triangle --steps 1 --warmup 1 --scale $SCALE --no-cpu > $OUT/bench_fetch.json 2> $OUT/fetch.log
timeout -k 10 300 rocprofv3 --kernel-include-regex "tri_" --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- python3 bench.py --query triangle --steps 1 --warmup 1 --scale $SCALE --no-cpu > $OUT/bench_write.json 2> $OUT/write.log
python3 tools/make_pmc_json.py $OUT $SCALE tri_
echo done
