#!/bin/bash
# Triangle s24 sweep: pass-A q-tile size (CAPF_TRI_QTILE) and pass-B p-block
# (CAPF_TRI_PBLOCK); one bench per setting, each under its own limit.
set -e
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --query triangle --steps 3 --warmup 1 --no-cpu > gpurun_out/tri_$n.json 2> gpurun_out/tri_$n.err
  python3 -c "import json;j=json.load(open('gpurun_out/tri_$n.json'));r=j['roofline'];print('$n', round(j['ms_per_step'],1), {k: round(v,1) for k,v in r['kernel_ms_per_query'].items()}, round(j['config']['first_query_ms']), j['config']['parity']['match'])"
}
run q0 CAPF_TRI_QTILE=0
run q23 CAPF_TRI_QTILE=23
run q24 CAPF_TRI_QTILE=24
run q25 CAPF_TRI_QTILE=25
run q26 CAPF_TRI_QTILE=26
run q25p22 CAPF_TRI_QTILE=25 CAPF_TRI_PBLOCK=22
run q25p23 CAPF_TRI_QTILE=25 CAPF_TRI_PBLOCK=23
run q25p25 CAPF_TRI_QTILE=25 CAPF_TRI_PBLOCK=25
