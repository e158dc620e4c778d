# rocprof kernel trace of the var2 rows leg (not a test): bench line + per-kernel stats
#   tools/prof_var2.sh [scale] [tag]
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SCALE=${1:-14}
TAG=${2:-var2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 240 python3 bench.py --query var2_rows --scale $SCALE --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o var2 --output-format csv -- python3 bench.py --query var2_rows --scale $SCALE --steps 10 --warmup 2 > $OUT/bench_traced.json 2> $OUT/trace.log
echo done
