# Config-2 PMC traffic (not a test): FETCH_SIZE / WRITE_SIZE passes over the
# per-query kernels of bench.py --query one_hop_person → gpurun_out/prof_c2/pmc_c2_s22.json
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_c2
mkdir -p $OUT
RE="c5_shard_partition|c5_bits_count|signed_terms"
timeout -k 10 300 rocprofv3 --kernel-include-regex "$RE" --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 bench.py --query one_hop_person --scale 22 --steps 5 --warmup 2 > $OUT/bench_fetch.json 2> $OUT/fetch.log
timeout -k 10 300 rocprofv3 --kernel-include-regex "$RE" --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- python3 bench.py --query one_hop_person --scale 22 --steps 5 --warmup 2 > $OUT/bench_write.json 2> $OUT/write.log
python3 tools/make_pmc_json.py $OUT 22 c2_
echo done
