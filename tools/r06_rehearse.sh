#!/bin/bash
# Multi-rank rehearsal of `bench.py --gpus N` on a one-GPU box (all ranks on
# cuda:0, gloo collectives): the N > 1 code path, not a scaling number.
set -e
mkdir -p gpurun_out
timeout -k 10 240 python -u bench.py --gpus 2 --one-device --steps 3 --warmup 1 --no-cpu --scale 22 \
  > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
timeout -k 10 300 python -u bench.py --gpus 8 --one-device --steps 3 --warmup 1 --no-cpu --scale 20 \
  > gpurun_out/rehearse8.json 2> gpurun_out/rehearse8.err
timeout -k 10 240 python -u bench.py --gpus 2 --one-device --layout edge --steps 3 --warmup 1 --no-cpu --scale 22 \
  > gpurun_out/rehearse2e.json 2> gpurun_out/rehearse2e.err
for f in rehearse2 rehearse8 rehearse2e; do python3 -c "import json,sys;d=json.load(open('gpurun_out/$f.json'));print('$f', d['n_gpus'], d['ms_per_step'], d['value'], d['config'].get('parallelism'))"; done
