# config 5 count kernel A/B: bit-sliced coalesced (default) vs ballot transpose (not a test)
set -e
timeout -k 10 400 python -u -m pytest tests/test_var_length_reach.py tests/test_ldbc_config5.py -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/vr_tests.log 2>&1
tail -1 gpurun_out/vr_tests.log
CAPF_VR_COUNT=0 timeout -k 10 300 python3 tools/config5_timing.py > gpurun_out/c5_old.txt 2>&1
timeout -k 10 300 python3 tools/config5_timing.py > gpurun_out/c5_new.txt 2>&1
tail -4 gpurun_out/c5_old.txt; tail -4 gpurun_out/c5_new.txt
