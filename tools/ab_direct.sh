# A/B of the default transpose-free 2-hop pipeline against the transpose pipeline (CAPF_C5_DIRECT=0) (not a test)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
CAPF_C5_DIRECT=0 bash tools/gpu_tests.sh ab_direct_tests tests/test_gpu_parity.py tests/test_headline_sizes.py -m gpu -q -k "two_hop or headline or chain2"
for i in 1 2; do
  CAPF_C5_DIRECT=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab/base_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab/direct_$i.json 2>/dev/null
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/trace -o direct --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ab/direct_traced.json 2> gpurun_out/ab/trace.log
for f in base_1 direct_1 base_2 direct_2; do python3 -c "
import json;d=json.load(open('gpurun_out/ab/$f.json'));c=d['config'];r=d['roofline']
print('$f', round(d['ms_per_step'],4), round(c['ms_per_step_pipelined'],4), round(r['pipeline_ms_per_query'],4), {k: round(v,4) for k,v in r['kernel_ms_per_query'].items()}, c['parity']['match'])"; done
