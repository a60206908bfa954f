#!/bin/bash
# Schedule knobs re-checked on the adapted window (iterations after 300 amcmc adaptation iterations):
# 32-subset shard (8-GPU share) and the 250-subset lookahead question.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k
mkdir -p $O
for v in "def MK_NONE=0" "mask16 MK_LA_MASK=16" "mask48 MK_LA_MASK=48" "mask64 MK_LA_MASK=64" "depth1 MK_CHOL_DEPTH=1" \
         "depth3 MK_CHOL_DEPTH=3" "thresh512 MK_TILE_THRESH=512" "head5 MK_LA_HEAD=5" "rows MK_SWEEP=5" "def2 MK_NONE=1"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32_$1.json 2> $O/b32_$1.err || exit 1
  echo "b32 $1 done"
done
for v in "def MK_NONE=0" "la MK_LOOKAHEAD=1"; do
  set -- $v
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/b250_$1.json 2> $O/b250_$1.err || exit 1
  echo "b250 $1 done"
done
timeout -k 10 120 python tools/dgemm_ceiling.py > $O/dgemm_ceiling.json 2> $O/dgemm_ceiling.err || exit 1
