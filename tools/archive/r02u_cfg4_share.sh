#!/bin/bash
# configs[3] per-GPU share on 8 GPUs (7 subsets of 2000, q = 3): default vs forced cooperative sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02u
mkdir -p $O
for v in "base X=0" "mg MK_SWEEP=2" "seq MK_LOOKAHEAD=0" "seqmg MK_LOOKAHEAD=0"; do
  set -- $v
  env $2 timeout -k 10 200 python run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 6 > $O/$1.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 1 --batch-length 30 > $O/tr.log 2>&1 || exit 1
