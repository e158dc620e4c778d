# var-length reach tests + config 5 timing (not a test)
set -e
timeout -k 10 400 python -u -m pytest tests/test_var_length_reach.py tests/test_ldbc_config5.py tests/test_gpu_parity.py -x -q -k "reach or var or config5 or ldbc or Bounded" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1
tail -2 gpurun_out/tests.log
timeout -k 10 300 python3 tools/config5_timing.py > gpurun_out/config5.txt 2>&1
head -4 gpurun_out/config5.txt
