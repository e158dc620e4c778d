#!/bin/bash
# Unique-build radix join (k_rj_direct): join parity tests, then the forced-radix
# sparse rows leg at s22 (tools/radix_sparse.sh).
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh rj_direct tests/test_gpu_parity.py tests/test_dense_join.py -m gpu -q -k "${TESTS_K:-radix or join or reference_case}"
SCALES=${SCALES:-22} bash tools/radix_sparse.sh
