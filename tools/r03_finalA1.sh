#!/bin/bash
# Round-3 closing pass: full gpu suite + smoke.
set -e
mkdir -p gpurun_out/final
F=gpurun_out/final
T="timeout -k 10"
echo "suite"; $T 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gputests.txt 2>&1
echo "smoke"; $T 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.txt 2>&1
echo done
