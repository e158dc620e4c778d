# kernel trace of the s24 2-hop count (FOR32, default variant): per-kernel
# durations and the gaps between them inside one query
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trace
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/trace -o run --output-format csv -- python3 tools/prof_chain2.py 24 ${1:-c4w} 1 > gpurun_out/trace/log.txt 2>&1
echo done
