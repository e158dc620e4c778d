# rocprof kernel trace of the materialising join leg (not a test), with the
# planner's join choice and with the radix join forced (CAPF_JOIN=radix)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_rows
mkdir -p $OUT
SCALE=${1:-22}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/auto -o rows --output-format csv -- python3 bench.py --query one_hop_rows --scale $SCALE --steps 5 --warmup 2 > $OUT/bench_auto.json 2> $OUT/trace_auto.log
CAPF_JOIN=radix timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/radix -o rows --output-format csv -- python3 bench.py --query one_hop_rows --scale $SCALE --steps 5 --warmup 2 > $OUT/bench_radix.json 2> $OUT/trace_radix.log
echo done
