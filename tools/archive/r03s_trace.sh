#!/bin/bash
# Kernel trace of the 32-subset shard (lookahead schedule) after the diagonal-tile rework.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr32 -o run -- python3 bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --adapt-batches 1 --no-kernel-events > $O/tr32.log 2>&1 || exit 1
python3 tools/stream_timeline.py $O/tr32/run_results.db 60 4 > $O/timeline32.txt 2>&1 || exit 1
