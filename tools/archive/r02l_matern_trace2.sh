#!/bin/bash
# Chebyshev-table range test + a short configs[1] kernel trace (lookahead schedule).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_linalg.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/la -o run -- python3 run_metakriging.py --config 2 --n-batch 1 --batch-length 40 > $O/la.log 2>&1 || exit 1
