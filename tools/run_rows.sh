# dense-join tests + rows leg (not a test)
set -e
timeout -k 10 300 python -u -m pytest tests/test_dense_join.py tests/test_gpu_parity.py -x -q -k "join or reference_case" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1
tail -2 gpurun_out/tests.log
timeout -k 10 120 python bench.py --query one_hop_rows --scale 22 --steps 10 --warmup 2 > gpurun_out/rows22.json 2>/dev/null
python3 -c "
import json;d=json.load(open('gpurun_out/rows22.json'));print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['timed_kernels_ms_per_step'])"
