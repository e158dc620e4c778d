# A/B of the P1 load schedule at s24 (not a test): CAPF_P1_UPFRONT=0/1, twice each
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "two_hop or headline or chain2" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1
tail -2 gpurun_out/tests.log
for u in 0 1 0 1; do
  CAPF_P1_UPFRONT=$u timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b_upf$u.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/b_upf$u.json'));r=d['roofline'];print($u, d['ms_per_step'], r['pipeline_ms_per_query'], r['kernel_ms_per_query']['c5_partition'], r['frac'])"
done
