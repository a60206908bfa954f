#!/bin/bash
# Kriging stream CU mask (MK_LA_KRIG_MASK) A/B at 32 and 63 subsets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02zc
mkdir -p $O
for r in 1 2; do
  for v in "m1 MK_LA_KRIG_MASK=1" "m0 MK_LA_KRIG_MASK=0"; do
    set -- $v
    env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32_$1_$r.json 2> $O/b32_$1_$r.err || exit 1
    env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --n 126000 --subsets 63 --steps 40 --warmup 4 > $O/b63_$1_$r.json 2> $O/b63_$1_$r.err || exit 1
  done
done
