#!/bin/bash
# round-6 GPU step: the -m gpu suite, then the triangle ILP 4 / ILP 3 A/B at s24
# (each under its own limit; stops on a timeout, abort or fault)
bash tools/gpu_tests.sh r06_suite tests -m gpu -q
rc=$?
echo "suite rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
for ilp in 4 3; do
  CAPF_TRI_ILP=$ilp timeout -k 10 300 python bench.py --query triangle --scale 24 --steps 5 --warmup 1 --no-cpu \
    > gpurun_out/r06_tri_ilp$ilp.json 2> gpurun_out/r06_tri_ilp$ilp.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_tri_ilp$ilp.json'));r=d['roofline'];print('ilp $ilp', d['ms_per_step'], r['kernel_ms_per_query'], r['frac'])"
done
