#!/bin/bash
# k_sweep_rows (MK_SWEEP=5) bit identity and speed, then the round's measurement pass.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_linalg.py -k bit_identical -x -v --timeout 280 --timeout-method thread > $O/bitid.log 2>&1 || exit 1
for v in "b32_one MK_SWEEP=1" "b32_rows MK_SWEEP=5"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/$1.json 2> $O/$1.err || exit 1
done
for v in "b250_one MK_SWEEP=1" "b250_rows MK_SWEEP=5"; do
  set -- $v
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/$1.json 2> $O/$1.err || exit 1
done
