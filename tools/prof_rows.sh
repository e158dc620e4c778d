# rocprof kernel trace of the materialising join leg (not a test)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_rows
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o rows --output-format csv -- python3 bench.py --query one_hop_rows --scale 20 --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/trace.log
echo done
