#!/bin/bash
# GPU suite twice + smoke + default bench (stability check of the committed state).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests1.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests2.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit 1
