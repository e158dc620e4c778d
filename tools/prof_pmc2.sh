# PMC passes on the partition kernels of the s24 2-hop (FOR32, default variant)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc2
V=${1:-c4w}
R="c4_|c3_"
i=0
for set in "SQ_WAVES SQ_INSTS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" ; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --kernel-include-regex "$R" --pmc $set -d gpurun_out/pmc2/p$i --output-format csv -- python3 tools/prof_chain2.py 24 $V 1 > gpurun_out/pmc2/log$i.txt 2>&1
done
echo done
