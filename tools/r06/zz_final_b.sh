#!/bin/bash
# round 6 final pass (part b): rocprofv3 kernel stats of the headline command, then part c (the PMC
# passes for the column-update traffic and the kriging GEMM, a 32-subset kernel trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r06fin}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof250 -o prof -- python3 -u bench.py --no-legs --no-e2e --no-cpu-baseline > $O/prof250.json 2> $O/prof250.log || { echo "prof failed"; tail -30 $O/prof250.log; exit 1; }
python3 tools/db_stats.py $O/prof250/prof_results.db > $O/kernel_stats_250.csv 2>&1 || { ls -R $O/prof250 | head; exit 1; }
head -4 $O/kernel_stats_250.csv
bash tools/r06/zz_final_c.sh || exit 1
