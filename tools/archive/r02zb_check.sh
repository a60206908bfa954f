#!/bin/bash
# Multi-workgroup sweep under lookahead on the unmasked session stream (q >= 2 small shards):
# GPU suite three times, configs[3] 8-GPU share timing.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02zb
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 240 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread > $O/gpu_tests$r.log 2>&1 || exit 1
done
timeout -k 10 120 python run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 6 > $O/c4_7.log 2>&1 || exit 1
timeout -k 10 120 python run_metakriging.py --config 4 --n 26000 --subsets 13 --n-batch 6 > $O/c4_13.log 2>&1 || exit 1
