#!/bin/bash
# Kernel traces of configs[1] (Matern, 50 subsets of 1000), 30 iterations, both schedules.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/la -o run -- python3 run_metakriging.py --config 2 --n-batch 1 --batch-length 40 > $O/la.log 2>&1 || exit 1
MK_LOOKAHEAD=0 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/seq -o run -- python3 run_metakriging.py --config 2 --n-batch 1 --batch-length 40 > $O/seq.log 2>&1 || exit 1
