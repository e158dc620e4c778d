# A/B of the sharded P1 load schedule (not a test): CAPF_SHARD_UPF=0/1 at G=2 and G=8
set -e
timeout -k 10 300 python -u -m pytest tests/test_headline_sizes.py tests/test_gpu_parity.py -x -q -k "node_partitioned or sharded" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1
tail -2 gpurun_out/tests.log
for g in 2 8; do for u in 0 1; do
  CAPF_SHARD_UPF=$u timeout -k 10 200 python tools/shard_timing.py 24 $g > gpurun_out/shard_g${g}_upf$u.txt 2>&1
  grep part gpurun_out/shard_g${g}_upf$u.txt | sed -E "s/.*(part [0-9]).*dev ([0-9.]+) ms.*'c5_gather': ([0-9.]+), 'c5_partition': ([0-9.]+).*/G=$g upf=$u \1 dev \2 P3 \3 P1 \4/"
  tail -1 gpurun_out/shard_g${g}_upf$u.txt
done; done
