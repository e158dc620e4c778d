# PMC passes over the fused 2-hop count (not a test).  Output: gpurun_out/pmc_p3/
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_p3
mkdir -p $OUT
RX="c5_partition|c5_gather"
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d $OUT/sq -o sq --output-format csv -- python3 tools/prof_variants.py 24 "" > $OUT/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$RX" --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 tools/prof_variants.py 24 "" > $OUT/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$RX" --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/tcc -o t --output-format csv -- python3 tools/prof_variants.py 24 "" > $OUT/tcc.log 2>&1
echo done
