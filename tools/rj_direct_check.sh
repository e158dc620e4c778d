#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh rj_direct tests/test_gpu_parity.py tests/test_dense_join.py -m gpu -q -k "radix or join or reference_case"
SCALES=22 bash tools/radix_sparse.sh
