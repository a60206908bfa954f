#!/bin/bash
# Diagonal tile with one barrier per step (next pivot beside the panel / inverse blocks): probe,
# GPU suite, windows at 32 and 250 subsets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03za
mkdir -p $O
timeout -k 10 60 ./tools/diag_probe 32 > $O/dp_32.log 2>&1 || exit 1
timeout -k 10 60 ./tools/diag_probe 250 > $O/dp_250.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32.json 2> $O/b32.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/b250.json 2> $O/b250.err || exit 1
