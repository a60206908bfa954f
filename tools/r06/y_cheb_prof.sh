#!/bin/bash
# round 6 (re-entry): kernel stats of two tiles of configs[4]'s per-GPU share (phi-interpolated kriging)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06y
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/cfg5_share.py --tiles 0:2 > $O/share.json 2> $O/share.err || { echo "prof failed"; tail -20 $O/share.err; exit 1; }
python3 tools/db_stats.py $O/prof/run_results.db > $O/kernel_stats.csv 2>&1 || { echo "db_stats failed"; tail $O/kernel_stats.csv; exit 1; }
head -25 $O/kernel_stats.csv
rm -rf $O/prof
