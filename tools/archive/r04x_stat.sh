#!/bin/bash
# Round 4: Monte Carlo-error parity tests (configs[1], configs[2], configs[3] geometry) on the GPU.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_stat_cfg2_cfg4.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/stat.log 2>&1 || { echo "stat rc $?"; tail -30 $O/stat.log; exit 1; }
tail -8 $O/stat.log
