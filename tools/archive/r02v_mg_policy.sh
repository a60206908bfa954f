#!/bin/bash
# Cooperative sweep under the lookahead schedule (MK_SWEEP=2) vs the one-workgroup default, by shard.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02v
mkdir -p $O
for v in "b32 X=0" "b32mg MK_SWEEP=2"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/$1.json 2> $O/$1.err || exit 1
done
for v in "c2 X=0" "c2mg MK_SWEEP=2"; do
  set -- $v
  env $2 timeout -k 10 200 python run_metakriging.py --config 2 --n-batch 10 > $O/$1.log 2>&1 || exit 1
done
for K in 13 25; do
  for v in "c4_$K X=0" "c4_${K}mg MK_SWEEP=2"; do
    set -- $v
    env $2 timeout -k 10 200 python run_metakriging.py --config 4 --n $((K * 2000)) --subsets $K --n-batch 6 > $O/$1.log 2>&1 || exit 1
  done
done
