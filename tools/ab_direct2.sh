# A/B: transpose-free pipeline with the XCD-grouped tile order (RM 1) vs the natural order (RM 2)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab2
CAPF_C5_DIRECT=1 CAPF_C5_RM=2 bash tools/gpu_tests.sh ab2_tests tests/test_headline_sizes.py -m gpu -q
for i in 1 2; do
  CAPF_C5_DIRECT=1 CAPF_C5_RM=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab2/rm1_$i.json 2>/dev/null
  CAPF_C5_DIRECT=1 CAPF_C5_RM=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab2/rm2_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab2/base_$i.json 2>/dev/null
done
for f in rm1_1 rm2_1 base_1 rm1_2 rm2_2 base_2; do python3 -c "
import json;d=json.load(open('gpurun_out/ab2/$f.json'));c=d['config'];r=d['roofline']
print('$f', round(d['ms_per_step'],4), round(c['ms_per_step_pipelined'],4), round(r['pipeline_ms_per_query'],4), {k: round(v,4) for k,v in r['kernel_ms_per_query'].items()}, c['parity']['match'])"; done
