set -e
bash tools/gpu_tests.sh r06_tri2 tests/test_headline_sizes.py tests/test_gpu_parity.py -m gpu -k "triangle or Triangle"
for v in "default" "CAPF_TRI_ILP=3" "CAPF_TRI_WPE=7" "CAPF_TRI_WPE=6" "default2"; do
  case $v in default*) unset CAPF_TRI_ILP CAPF_TRI_WPE;; *) export $v;; esac
  timeout -k 10 300 python -u bench.py --query triangle --steps 5 --warmup 2 --no-cpu > gpurun_out/tri_$v.json 2> gpurun_out/tri_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/tri_$v.json'));print('$v', d['ms_per_step'], d['roofline']['frac'])"
  unset CAPF_TRI_ILP CAPF_TRI_WPE
done
