#!/bin/bash
# configs[3]'s 8-GPU share (7 subsets, q = 3): per-kernel stats and one iteration's stream timeline,
# split-launch sweep (default) and the one-workgroup sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/q3step -o run -- python3 run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 6 > $O/q3step.log 2>&1 || exit 1
MK_SWEEP=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/q3one -o run -- python3 run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 6 > $O/q3one.log 2>&1 || exit 1
timeout -k 10 120 ./tools/gemm_probe2 > $O/gemm_probe2.log 2>&1 || exit 1
