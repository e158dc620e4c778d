timeout -k 10 200 python3 tools/prof_variants.py 24 "" "CAPF_P3_HOT=1" "CAPF_P3_HOT=1;CAPF_P3_DEPTH=2" "CAPF_P3_DEPTH=2" > gpurun_out/r2_var5.txt 2>&1
rm -f gpurun_out/p3trace3.bin
CAPF_P3_HOT=1 CAPF_P3_TRACE=gpurun_out/p3trace3.bin timeout -k 10 100 python3 tools/prof_variants.py 24 "" >> gpurun_out/r2_var5.txt 2>&1
python3 tools/p3_trace.py gpurun_out/p3trace3.bin >> gpurun_out/r2_var5.txt 2>&1
echo done
