# Config 2 semi-join A/B (not a test): row-by-row bitmap probes vs radix-partitioned
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_headline_sizes.py -x -q -k "person" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1
tail -2 gpurun_out/tests.log
for u in 0 1; do
  CAPF_SEMI_PART=$u timeout -k 10 200 python bench.py --query one_hop_person --scale 22 --steps 20 --warmup 3 --no-cpu > gpurun_out/person_semi$u.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/person_semi$u.json'));r=d['roofline'];print($u, d['ms_per_step'], r['pipeline_ms_per_query'], r['kernel_ms_per_query'], r['end_to_end_frac'], d['config']['parity'])"
done
