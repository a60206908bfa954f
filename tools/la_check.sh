#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/la
mkdir -p $O
echo "box GPU_MAX_HW_QUEUES=$GPU_MAX_HW_QUEUES" > $O/env.log
B="python bench.py --no-cpu-baseline"
for K in 32 63 125 250; do
  timeout -k 10 200 $B --n $((K * 2000)) --subsets $K > $O/b$K.log 2>&1 || exit 1
done
