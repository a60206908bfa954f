#!/bin/bash
# diagonal tile: next trailing block on wave 0 in phase 2, trailing blocks four at a time
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 60 ./tools/diag_probe 32 > $O/dp_32.log 2>&1 || exit 1
timeout -k 10 60 ./tools/diag_probe 250 > $O/dp_250.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32.json 2> $O/b32.err || exit 1
