#!/bin/bash
# Kernel trace of the 32-subset shard (lookahead schedule) for the per-iteration critical path.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr32 -o run -- python3 bench.py --no-cpu-baseline --n 64000 --subsets 32 --no-kernel-events > $O/tr32.log 2>&1 || exit 1
