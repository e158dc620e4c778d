#!/bin/bash
# round-6 GPU step: the tail of the -m gpu suite, then the triangle waves-per-SIMD A/B at s24
bash tools/gpu_tests.sh r06_tail2 tests/test_jni_exec.py tests/test_ldbc_config5.py tests/test_string_functions.py \
  tests/test_var_length_reach.py -m gpu
rc=$?
echo "tail rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
for w in 6 7 8; do
  CAPF_TRI_WPE=$w timeout -k 10 300 python bench.py --query triangle --scale 24 --steps 5 --warmup 1 --no-cpu \
    > gpurun_out/r06_tri_wpe$w.json 2> gpurun_out/r06_tri_wpe$w.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_tri_wpe$w.json'));r=d['roofline'];print('wpe $w', d['ms_per_step'], r['kernel_ms_per_query'], r['frac'], d['config']['parity'])"
done
