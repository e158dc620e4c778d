#!/bin/bash
# Round-3 GPU pass at HEAD: new tests, smoke, default bench, triangle / rows legs, profiles, full gpu suite.
set -e
mkdir -p gpurun_out
T="timeout -k 10"
echo "new tests"; $T 900 python -u -m pytest tests/test_dense_join.py tests/test_fs_source.py "tests/test_gpu_parity.py::test_triangle_heavy_multi_edges" "tests/test_gpu_parity.py::test_triangle_count_rmat" tests/test_headline_sizes.py tests/test_dist_gpu.py -k "triangle or hashed or sparse or nullable or dense or partitioned or dist" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_newtests.txt 2>&1
echo "smoke"; $T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.txt 2>&1
echo "bench"; $T 400 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err
echo "tri packed ilp4"; $T 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/r03_tri_p4.json 2> gpurun_out/r03_tri_p4.err
echo "tri packed ilp2"; CAPF_TRI_ILP=2 $T 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/r03_tri_p2.json 2> gpurun_out/r03_tri_p2.err
echo "tri unpacked"; CAPF_TRI_PACKED=0 $T 300 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/r03_tri_u4.json 2> gpurun_out/r03_tri_u4.err
echo "rows sparse"; $T 300 python -u bench.py --query one_hop_rows --scale 22 --steps 10 --warmup 3 --id-stride 1000003 > gpurun_out/r03_rows_sparse.json 2> gpurun_out/r03_rows_sparse.err
echo "rows sparse radix"; CAPF_JOIN=radix $T 300 python -u bench.py --query one_hop_rows --scale 22 --steps 5 --warmup 2 --id-stride 1000003 > gpurun_out/r03_rows_sparse_radix.json 2> gpurun_out/r03_rows_sparse_radix.err
echo "shard g8"; $T 300 python -u tools/shard_timing.py 24 8 > gpurun_out/r03_shard_g8_s24.txt 2>&1
echo "shard g8 untrusted"; CAPF_SHARD_TRUST=0 $T 300 python -u tools/shard_timing.py 24 8 > gpurun_out/r03_shard_g8_s24_untrusted.txt 2>&1
echo "shard g8 tile24"; CAPF_SHARD_TILE=24 $T 300 python -u tools/shard_timing.py 24 8 > gpurun_out/r03_shard_g8_s24_t24.txt 2>&1
echo "profiles"; bash tools/collect_profiles.sh 24 > gpurun_out/r03_collect.txt 2>&1
echo "full suite"; $T 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gputests.txt 2>&1
echo done
