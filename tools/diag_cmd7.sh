timeout -k 10 200 python3 tools/prof_variants.py 24 "" "CAPF_P3_LPT=1" "CAPF_P3_LPT=1;CAPF_P3_SPLIT=1.2" "CAPF_P3_LPT=1;CAPF_P3_SPLIT=1.15;CAPF_P3_DEPTH=2" "CAPF_P3_SPLIT=1.2" > gpurun_out/r2_var4.txt 2>&1
rm -f gpurun_out/p3trace2.bin
CAPF_P3_LPT=1 CAPF_P3_SPLIT=1.2 CAPF_P3_TRACE=gpurun_out/p3trace2.bin timeout -k 10 100 python3 tools/prof_variants.py 24 "" >> gpurun_out/r2_var4.txt 2>&1
python3 tools/p3_trace.py gpurun_out/p3trace2.bin >> gpurun_out/r2_var4.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CAPF_P3_LPT=1 CAPF_P3_SPLIT=1.2 timeout -s KILL 90 rocprofv3 --kernel-include-regex "c5_gather" --pmc FETCH_SIZE -d gpurun_out/r2fetch_lpt -o f --output-format csv -- python3 tools/prof_variants.py 24 "" > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --kernel-include-regex "c5_gather" --pmc FETCH_SIZE -d gpurun_out/r2fetch_base -o f --output-format csv -- python3 tools/prof_variants.py 24 "" > /dev/null 2>&1
echo done
