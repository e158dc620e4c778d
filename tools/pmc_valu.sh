# PMC pass over the fused 2-hop count: instruction mix (not a test).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_valu
mkdir -p $OUT
RX="c5_partition|c5_gather"
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $OUT/a -o a --output-format csv -- python3 tools/prof_variants.py 24 "" > $OUT/a.log 2>&1
echo done
