#!/bin/bash
# Round-3 GPU pass at HEAD: new tests, smoke, default bench, rows legs, profiles, full gpu suite.
set -e
mkdir -p gpurun_out
echo "new tests"; timeout -k 10 600 python -u -m pytest tests/test_dense_join.py tests/test_fs_source.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_newtests.txt 2>&1
echo "smoke"; timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.txt 2>&1
echo "bench"; timeout -k 10 400 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err
echo "rows sparse"; timeout -k 10 300 python -u bench.py --query one_hop_rows --scale 22 --steps 10 --warmup 3 --id-stride 1000003 > gpurun_out/r03_rows_sparse.json 2> gpurun_out/r03_rows_sparse.err
echo "rows sparse radix"; CAPF_JOIN=radix timeout -k 10 300 python -u bench.py --query one_hop_rows --scale 22 --steps 5 --warmup 2 --id-stride 1000003 > gpurun_out/r03_rows_sparse_radix.json 2> gpurun_out/r03_rows_sparse_radix.err
echo "profiles"; bash tools/collect_profiles.sh 24 > gpurun_out/r03_collect.txt 2>&1
echo "full suite"; timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gputests.txt 2>&1
echo done
