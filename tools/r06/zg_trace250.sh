#!/bin/bash
# round 6 (re-entry): a 250-subset kernel trace (burn-in and kept iterations of the bench window)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zg
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr250 -o run -- python3 bench.py --no-legs --no-cpu-baseline --no-e2e --steps 20 --no-kernel-events > $O/tr250.json 2> $O/tr250.log || { echo "trace failed"; tail $O/tr250.log; exit 1; }
python3 tools/stream_timeline.py $O/tr250/run_results.db 310 1 > $O/timeline250_burnin_310.txt 2>&1 || exit 1
python3 tools/stream_timeline.py $O/tr250/run_results.db 320 1 > $O/timeline250_kept_320.txt 2>&1 || exit 1
rm -rf $O/tr250
head -3 $O/timeline250_burnin_310.txt | cut -c1-300
