#!/bin/bash
# Node driver tests, then the split-launch sweep (MK_SWEEP=3, default for q >= 2 on <= 16 subsets)
# against the one-workgroup sweep (MK_SWEEP=1) on configs[3]'s 8-GPU share and a q = 1 32-subset shard.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_node.py -x -v --timeout 120 --timeout-method thread > $O/node_tests.log 2>&1 || exit 1
for K in 7 13; do
  for v in "c4_${K}_one MK_SWEEP=1" "c4_${K}_split MK_SWEEP=0"; do
    set -- $v
    env $2 timeout -k 10 200 python run_metakriging.py --config 4 --n $((K * 2000)) --subsets $K --n-batch 6 > $O/$1.log 2>&1 || exit 1
  done
done
for v in "b32_one MK_SWEEP=1" "b32_split MK_SWEEP=3"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/$1.json 2> $O/$1.err || exit 1
done
