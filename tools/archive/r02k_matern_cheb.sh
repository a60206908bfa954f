#!/bin/bash
# Matern Chebyshev tables: GPU tests, then configs[1] end to end.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02m
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python run_metakriging.py --config 2 > $O/e2e_cfg2.log 2>&1 || exit 1
