#!/bin/bash
# Round 4: the GPU suite with the stream pool's eviction, then the bench's legs in one process.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite rc $?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
O=$O bash tools/r04p_legs.sh
