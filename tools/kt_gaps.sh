# kernel trace of the s24 bench (not a test): per-query span vs busy time
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/kt -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/kt.json 2>/dev/null
echo done
