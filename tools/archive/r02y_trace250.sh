#!/bin/bash
# Kernel trace of the 250-subset sequential schedule (per-launch durations of the inverse levels).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02y
mkdir -p $O
MK_SWEEP=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 bench.py --no-cpu-baseline --no-kernel-events --steps 8 > $O/tr.log 2>&1 || exit 1
