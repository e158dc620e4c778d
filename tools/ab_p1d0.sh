# P1 FOR24 decode without mask/add (UPF 3) A/B at s24 (not a test)
set -e
run() {
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/x.json 2>/dev/null
  python3 -c "
import json,sys;d=json.load(open('gpurun_out/x.json'));r=d['roofline'];k=r['kernel_ms_per_query']
print(sys.argv[1:], round(d['ms_per_step'],4), round(r['pipeline_ms_per_query'],4), round(k['c5_gather'],4), round(k['c5_partition'],4), d['config']['parity']['match'])" "$@"
}
run CAPF_NONE=1
run CAPF_P1_UPFRONT=3
run CAPF_NONE=1
run CAPF_P1_UPFRONT=3
run CAPF_NONE=1
run CAPF_P1_UPFRONT=3
