#!/bin/bash
# Round-4 check: GPU tests from the distributed SPI test on, 2-rank bench rehearsal
# through the SPI, the s24 triangle pass-A q-tile sweep, host profile.
set -e
bash tools/gpu_tests.sh full3 tests/test_dist_gpu.py tests/test_edge_list.py tests/test_fs_source.py tests/test_gpu_parity.py tests/test_headline_sizes.py tests/test_jni_shim.py tests/test_ldbc_config5.py tests/test_var_length_reach.py -m gpu -q
timeout -k 10 300 python -u bench.py --gpus 2 --one-device --scale 20 --steps 5 --warmup 2 > gpurun_out/dist2.json 2> gpurun_out/dist2.err
for qt in 0 20 22 24; do
  CAPF_TRI_QTILE=$qt timeout -k 10 300 python -u bench.py --query triangle --steps 3 --warmup 1 --no-cpu > gpurun_out/tri_q$qt.json 2> gpurun_out/tri_q$qt.err
  python3 -c "import json;j=json.load(open('gpurun_out/tri_q$qt.json'));print('qtile $qt', j['ms_per_step'], j['config']['first_query_ms'], j['config']['parity'])"
done
CAPF_HOST_TRACE=1 timeout -k 10 300 python -u tools/prof_host.py 24 > gpurun_out/prof_host_s24.txt 2>&1
