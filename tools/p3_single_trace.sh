# per-unit P3 timeline of the single-GPU s24 pipeline (not a test)
set -e
CAPF_P3_TRACE=gpurun_out/p3.bin timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --sync-steps > /dev/null 2>&1
python3 tools/p3_trace.py gpurun_out/p3.bin > gpurun_out/p3.txt
cat gpurun_out/p3.txt
