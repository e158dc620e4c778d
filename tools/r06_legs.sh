#!/bin/bash
# Round-6 re-measurement of the non-headline bench legs at the closing build
# (each under its own limit; stops at the first failure).
set -e
mkdir -p gpurun_out/legs
run() { name=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/legs/$name.json 2> gpurun_out/legs/$name.err; \
  python3 -c "import json;d=json.load(open('gpurun_out/legs/$name.json'));r=d.get('roofline') or {};print('$name', d['ms_per_step'], r.get('frac'), (d.get('cpu_baseline') or {}).get('value'))"; }
run config2_s22 --query one_hop_person --scale 22
run var2_rows_s14 --query var2_rows --scale 14
run rows_sparse_s22 --query one_hop_rows --scale 22 --id-stride 1000003
run reach_sf10 --query reach
run triangle_s24 --query triangle --steps 5 --warmup 2
