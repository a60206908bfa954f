#!/bin/bash
# GPU tests + default bench + 32-subset bench (interior-tile candidate path).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02q
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32.json 2> $O/b32.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof250 -o run -- python3 bench.py --no-cpu-baseline > $O/prof250.log 2>&1 || exit 1
