#!/bin/bash
# rocprofv3 kernel stats of the committed state at 250 and 32 subsets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03zf
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof250 -o run -- python3 bench.py --no-cpu-baseline --no-e2e > $O/prof250.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof32 -o run -- python3 bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 > $O/prof32.log 2>&1 || exit 1
