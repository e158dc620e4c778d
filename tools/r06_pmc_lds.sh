#!/bin/bash
# LDS counters of the headline's P1 / P3 kernels at the closing build (not a
# test): one SQ pass (8 counters) over the default bench → gpurun_out/pmc_lds/
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_lds
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-include-regex "c5_partition|c5_gather" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES -d $OUT/sq -o sq --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $OUT/sq.json 2> $OUT/sq.log
python3 - <<'P'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_lds/sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("capf::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k, {c: round(x) for c, x in sorted(avg.items())})
    if avg.get("SQ_LDS_IDX_ACTIVE"):
        print("  bank-conflict cycles / LDS-active cycles = %.3f" % (avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"]))
P
