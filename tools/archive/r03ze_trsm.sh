#!/bin/bash
# trsm row-block size A/B (MK_TRSM_TILE) at 250 and 32 subsets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ze
mkdir -p $O
for v in "def MK_NONE=0" "t64 MK_TRSM_TILE=64" "t32 MK_TRSM_TILE=32"; do
  set -- $v
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/b250_$1.json 2> $O/b250_$1.err || exit 1
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32_$1.json 2> $O/b32_$1.err || exit 1
  echo "$1 done"
done
