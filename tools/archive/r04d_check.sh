#!/bin/bash
# Round 4: the GPU suite once more (site sweep at one wave per SIMD), then the knob comparison.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite rc $?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/r04b_knobs.sh
