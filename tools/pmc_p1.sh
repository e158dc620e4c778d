# PMC of the single-GPU P1 vs the sharded P1 at G=2 (not a test): wave states,
# LDS issue / conflicts, VALU per dispatch.  One pass each, under a kill timer.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/p1pmc
mkdir -p $OUT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "c5_partition" --pmc $C -d $OUT/single -o s --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/single.json 2> $OUT/single.log
timeout -s KILL 150 rocprofv3 --kernel-include-regex "c5_shard_partition" --pmc $C -d $OUT/g2 -o g --output-format csv -- python3 tools/shard_timing.py 24 2 0 > $OUT/g2.txt 2> $OUT/g2.log
echo done
