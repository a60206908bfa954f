#!/bin/bash
# configs[3] (q = 3 LMC) short runs: default vs cooperative sweep vs sequential schedule.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02o
mkdir -p $O
for v in "base X=0" "mg MK_SWEEP=2" "seq MK_LOOKAHEAD=0" "base2 X=0"; do
  set -- $v
  env $2 timeout -k 10 200 python run_metakriging.py --config 4 --n-batch 6 > $O/$1.log 2>&1 || exit 1
done
