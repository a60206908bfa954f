#!/bin/bash
# Cooperative multi-workgroup sweep for q >= 2 small shards under lookahead: GPU suite twice,
# configs[3] 8-GPU share timing, smoke.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02za
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests1.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests2.log 2>&1 || exit 1
timeout -k 10 120 python run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 6 > $O/c4_7.log 2>&1 || exit 1
timeout -k 10 200 python run_metakriging.py --config 4 --n 14000 --subsets 7 > $O/e2e_cfg4_share8.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
