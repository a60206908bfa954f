#!/bin/bash
# Diagonal-tile kernel v2 (reciprocal-chain pivot, stores behind the pivot chain): probe A/B vs the
# old pivot, the GPU suite, then the 32- and 250-subset bench windows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 60 ./tools/diag_probe_v1 32 > $O/dp_v1_32.log 2>&1 || exit 1
timeout -k 10 60 ./tools/diag_probe 32 > $O/dp_v2_32.log 2>&1 || exit 1
timeout -k 10 60 ./tools/diag_probe 250 > $O/dp_v2_250.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32.json 2> $O/b32.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/b250.json 2> $O/b250.err || exit 1
