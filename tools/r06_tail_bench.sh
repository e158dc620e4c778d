#!/bin/bash
# round-6 GPU step: the tail of the -m gpu suite (after test_gpu_parity), then the default bench line
bash tools/gpu_tests.sh r06_tail tests/test_jni_exec.py tests/test_ldbc_config5.py tests/test_string_functions.py \
  tests/test_var_length_reach.py -m gpu
rc=$?
echo "tail rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py > gpurun_out/r06_bench2.json 2> gpurun_out/r06_bench2.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r06_bench2.json'));r=d['roofline'];print(d['ms_per_step'], r['frac'], r['kernel_event_frac'], d['config']['ms_per_step_pipelined'])"
