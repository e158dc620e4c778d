# round-end sanity of every bench leg (not a test)
set -e
timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/b2hop.json 2>/dev/null
timeout -k 10 300 python bench.py --gpus 2 --one-device --steps 5 --warmup 2 > gpurun_out/d2.json 2>gpurun_out/d2.err
timeout -k 10 300 python bench.py --gpus 2 --one-device --query triangle --scale 20 --steps 3 --warmup 1 > gpurun_out/d2tri.json 2>gpurun_out/d2tri.err
timeout -k 10 120 python bench.py --query one_hop_person --scale 22 --steps 20 --warmup 3 --no-cpu > gpurun_out/person.json 2>/dev/null
for f in b2hop d2 d2tri person; do python3 -c "
import json;d=json.load(open('gpurun_out/$f.json'));c=d['config'];print('$f', d['n_gpus'], round(d['ms_per_step'],3), c.get('count'), c.get('parity'), c.get('ms_per_query_median_plan_to_scalar'))"; done
