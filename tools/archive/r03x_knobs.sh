#!/bin/bash
# Schedule knobs re-checked at 32 subsets after the diagonal-tile rework (40-step windows).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03x
mkdir -p $O
for v in "def MK_NONE=0" "mask24 MK_LA_MASK=24" "mask40 MK_LA_MASK=40" "depth3 MK_CHOL_DEPTH=3" "thresh192 MK_TILE_THRESH=192" \
         "thresh384 MK_TILE_THRESH=384" "head2 MK_LA_HEAD=2" "head4 MK_LA_HEAD=4" "def2 MK_NONE=1"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32_$1.json 2> $O/b32_$1.err || exit 1
  echo "b32 $1 done"
done
