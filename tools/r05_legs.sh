# Round-5 bench legs beside the headline (not a test): triangle (with the Flink-shaped
# CPU baseline), forced-radix sparse rows leg, config 2
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/legs
timeout -k 10 400 python -u bench.py --query triangle --steps 3 --warmup 1 > gpurun_out/legs/triangle.json 2> gpurun_out/legs/triangle.err
CAPF_JOIN=radix timeout -k 10 300 python -u bench.py --query one_hop_rows --scale 22 --id-stride 1000003 --steps 10 --warmup 2 > gpurun_out/legs/rows_sparse_radix.json 2> gpurun_out/legs/rows_sparse_radix.err
timeout -k 10 300 python -u bench.py --query one_hop_rows --scale 22 --id-stride 1000003 --steps 10 --warmup 2 > gpurun_out/legs/rows_sparse.json 2> gpurun_out/legs/rows_sparse.err
timeout -k 10 300 python -u bench.py --query one_hop_person --scale 22 --steps 20 --warmup 3 > gpurun_out/legs/config2.json 2> gpurun_out/legs/config2.err
echo done
