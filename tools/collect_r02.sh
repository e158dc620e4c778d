# Round-2 profile collection on the GPU box (not a test).  Every step has its
# own time limit; the chain stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02
mkdir -p $O
# config 3 (headline): kernel trace + FETCH/WRITE PMC passes
bash tools/collect_profiles.sh 24
# config 2: bench line + kernel trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2 -o c2 --output-format csv -- python3 bench.py --query one_hop_person --scale 22 --steps 20 --warmup 3 --no-cpu > $O/bench_config2_s22.json 2> $O/c2.log
# config 4: trace + PMC bytes + PMC detail
bash tools/collect_tri_profiles.sh 24
bash tools/pmc_tri_detail.sh 22
# config 5: end-to-end timing + kernel split
timeout -k 10 300 python3 tools/config5_timing.py > $O/config5_sf10_timing.txt 2>&1
echo done
