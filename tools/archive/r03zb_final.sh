#!/bin/bash
# Round-3 last pass on the committed state: the GPU suite and smoke as the driver runs them, the
# default bench (window + CPU baseline + end-to-end leg).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03zb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
