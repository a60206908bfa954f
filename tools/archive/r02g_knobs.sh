#!/bin/bash
# Schedule-knob sweep at the 32-subset shard (the per-GPU share of configs[2] on 8 GPUs).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02g
mkdir -p $O
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/$lab.json 2> $O/$lab.err || exit 1
}
run base0 X=0
run mask64 MK_LA_MASK=64
run mask16 MK_LA_MASK=16
run res64 MK_RESERVE_CU=64
run mask64res64 MK_LA_MASK=64 MK_RESERVE_CU=64
run depth3 MK_CHOL_DEPTH=3
run depth1 MK_CHOL_DEPTH=1
run thr128 MK_TILE_THRESH=128
run thr512 MK_TILE_THRESH=512
run head5 MK_LA_HEAD=5
run head1 MK_LA_HEAD=1
run prio0 MK_LA_PRIO=0
run base1 X=0
