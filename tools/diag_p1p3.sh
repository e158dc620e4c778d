# Diagnostics of the fused 2-hop kernels (not a test): variant timings and
# LDS/VALU PMC passes over P1 (k_c5_partition) and P3 (k_c5_gather).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/diag
mkdir -p $OUT
timeout -k 10 120 python3 tools/prof_variants.py 24 "" "CAPF_P1_DIAG=1" "CAPF_P1_DIAG=2" "CAPF_P3_DIAG=2" > $OUT/variants.txt 2>&1
RX="c5_partition|c5_gather"
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT -d $OUT/sq1 -o sq --output-format csv -- python3 tools/prof_variants.py 24 "" > $OUT/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/sq2 -o sq --output-format csv -- python3 tools/prof_variants.py 24 "" > $OUT/sq2.log 2>&1
echo done
