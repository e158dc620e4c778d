set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for v in twopass single; do for c in 0 1; do
  timeout -k 10 180 rocprofv3 --kernel-include-regex "c2_|c3_" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc/sq_${v}_${c} --output-format csv -- python3 tools/prof_chain2.py 24 $v $c > gpurun_out/pmc/log_sq_${v}_${c}.txt 2>&1
  timeout -k 10 180 rocprofv3 --kernel-include-regex "c2_|c3_" --pmc FETCH_SIZE -d gpurun_out/pmc/fe_${v}_${c} --output-format csv -- python3 tools/prof_chain2.py 24 $v $c > gpurun_out/pmc/log_fe_${v}_${c}.txt 2>&1
  timeout -k 10 180 rocprofv3 --kernel-include-regex "c2_|c3_" --pmc WRITE_SIZE -d gpurun_out/pmc/wr_${v}_${c} --output-format csv -- python3 tools/prof_chain2.py 24 $v $c > gpurun_out/pmc/log_wr_${v}_${c}.txt 2>&1
done; done
echo done
