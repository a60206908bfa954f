#!/bin/bash
# GPU suite + smoke after pooling the node driver's per-block streams.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03zc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --e2e-only --e2e-devices 0,0 > $O/e2e_only_00.json 2> $O/e2e_only_00.err || exit 1
