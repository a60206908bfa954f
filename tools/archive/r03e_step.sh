#!/bin/bash
# k_sweep_step (one launch per block) vs the two-kernel split sweep and the one-workgroup sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_linalg.py -k bit_identical -x -v --timeout 300 --timeout-method thread > $O/bitid.log 2>&1 || exit 1
for K in 7 13; do
  for v in "c4_${K}_step MK_SWEEP=3" "c4_${K}_two MK_SWEEP=4"; do
    set -- $v
    env $2 timeout -k 10 200 python run_metakriging.py --config 4 --n $((K * 2000)) --subsets $K --n-batch 6 > $O/$1.log 2>&1 || exit 1
  done
done
for v in "b32_one MK_SWEEP=1" "b32_step MK_SWEEP=3"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/$1.json 2> $O/$1.err || exit 1
done
