#!/bin/bash
# Diagonal-tile store phase: probe + GPU tests + 32 / 250-subset benches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02t
mkdir -p $O
timeout -k 10 60 ./tools/diag_probe 32 > $O/diag_probe32.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32.json 2> $O/b32.err || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline > $O/b250.json 2> $O/b250.err || exit 1
