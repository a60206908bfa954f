#!/bin/bash
# Sweep policy (cooperative kernel for q >= 2 small shards under lookahead): GPU tests, configs[3]
# per-GPU shares and end to end.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02w
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
for K in 7 13; do
  timeout -k 10 200 python run_metakriging.py --config 4 --n $((K * 2000)) --subsets $K --n-batch 6 > $O/c4_$K.log 2>&1 || exit 1
done
timeout -k 10 300 python run_metakriging.py --config 4 --n 14000 --subsets 7 > $O/e2e_cfg4_share8.log 2>&1 || exit 1
