#!/bin/bash
# Round-3 closing measurement pass: GPU suite, smoke, the default bench (window + CPU baseline +
# end-to-end leg, what the driver runs), rocprofv3 kernel stats at 250 and 32 subsets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof250 -o run -- python3 bench.py --no-cpu-baseline --no-e2e > $O/prof250.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof32 -o run -- python3 bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 > $O/prof32.log 2>&1 || exit 1
