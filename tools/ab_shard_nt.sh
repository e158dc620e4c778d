# A/B of non-temporal loads in the sharded P1 ring (CAPF_SHARD_UPF=1 vs 2) at G=2 and G=8 (not a test)
set -e
CAPF_SHARD_UPF=2 timeout -k 10 300 python -u -m pytest tests/test_headline_sizes.py tests/test_gpu_parity.py -x -q -k "node_partitioned or sharded or chain2 or two_hop" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1
tail -2 gpurun_out/tests.log
for g in 2 8; do for u in 1 2 1 2; do
  CAPF_SHARD_UPF=$u timeout -k 10 200 python tools/shard_timing.py 24 $g > gpurun_out/shard_g${g}_upf$u.txt 2>&1
  python3 - gpurun_out/shard_g${g}_upf$u.txt $g $u <<'PY'
import re,sys
t=open(sys.argv[1]).read()
dev=[float(x) for x in re.findall(r'dev ([0-9.]+) ms',t)]
p1=[float(x) for x in re.findall(r"'c5_partition': ([0-9.]+)",t)]
print('G',sys.argv[2],'upf',sys.argv[3],'max dev',max(dev),'max P1',max(p1),'mean P1',round(sum(p1)/len(p1),4), t.strip().splitlines()[-1])
PY
done; done
