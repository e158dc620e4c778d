# PMC detail of the triangle count kernel (not a test): where k_tri_count's
# cycles go (wave states, LDS issue / bank conflicts) and its L2 hit rate.
# Each pass runs alone, under its own kill timer.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tpmc
mkdir -p $OUT
SCALE=${1:-22}
timeout -s KILL 120 rocprofv3 --kernel-include-regex tri_count --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD -d $OUT/sq -o sq --output-format csv -- python3 bench.py --query triangle --scale $SCALE --steps 1 --warmup 0 --no-cpu > $OUT/sq.json 2> $OUT/sq.log
timeout -s KILL 120 rocprofv3 --kernel-include-regex tri_count --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/tcc -o tcc --output-format csv -- python3 bench.py --query triangle --scale $SCALE --steps 1 --warmup 0 --no-cpu > $OUT/tcc.json 2> $OUT/tcc.log
echo done
