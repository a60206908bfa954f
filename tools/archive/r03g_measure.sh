#!/bin/bash
# Round-3 measurement pass (1/2): the GPU suite, smoke, the default bench (what the driver runs:
# window + CPU baseline + end-to-end leg), rocprofv3 kernel stats at 250 and 32 subsets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_default.log 2> $O/bench_default.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof250 -o run -- python3 bench.py --no-cpu-baseline --no-e2e > $O/prof250.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof32 -o run -- python3 bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 > $O/prof32.log 2>&1 || exit 1
