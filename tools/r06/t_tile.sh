#!/bin/bash
# round 6: the kriging tile clamp (mk_session_predict_tile) and the sampled-event test, plus the node tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_cfg5.py tests/test_gpu_errors.py tests/test_gpu_node.py tests/test_gpu_post.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
