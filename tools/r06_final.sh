#!/bin/bash
# Round-6 final measurement at the closing build (not a test): headline kernel
# trace + PMC, the leg PMC passes, then the bench lines (which read those PMC
# files) and smoke(); stops at the first failure.
set -e
bash tools/collect_profiles.sh 24 > gpurun_out/closing_prof.log 2>&1
cp gpurun_out/prof/pmc_s24.json profiles/pmc_s24.json
bash tools/collect_c2_pmc.sh > gpurun_out/c2pmc.log 2>&1
cp gpurun_out/prof_c2/pmc_c2_s22.json profiles/pmc_c2_s22.json
bash tools/collect_reach_profiles.sh > gpurun_out/rpmc.log 2>&1
cp gpurun_out/rprof/pmc_reach_s16.json profiles/pmc_reach_s16.json
bash tools/collect_tri_profiles.sh 24 > gpurun_out/tpmc.log 2>&1
cp gpurun_out/tprof/pmc_tri_s24.json profiles/pmc_tri_s24.json
bash tools/collect_rows_pmc.sh > gpurun_out/rows_pmc.log 2>&1
cp gpurun_out/prof_rows/pmc_rows_sparse_s22.json profiles/pmc_rows_sparse_s22.json
timeout -k 10 300 python -u bench.py > gpurun_out/closing_bench.json 2> gpurun_out/closing_bench.err
bash tools/r06_legs.sh
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/closing_smoke.log 2>&1
python3 -c "import json;d=json.load(open('gpurun_out/closing_bench.json'));r=d['roofline'];print('headline', d['ms_per_step'], r['frac'], r.get('kernel_event_frac'), r['traffic_source']['lib'], d['config'].get('lib'))"
tail -n 1 gpurun_out/closing_smoke.log
