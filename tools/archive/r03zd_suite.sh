#!/bin/bash
# GPU suite (with the stream-pool test) and smoke on the committed state.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03zd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
