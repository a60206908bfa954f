#!/bin/bash
# round 6 (re-entry): the phi-interpolation tests and the node tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ze
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_krig_cheb.py tests/test_gpu_node.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
