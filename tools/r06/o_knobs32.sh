#!/bin/bash
# round 6: the small-shard knobs re-checked at the 32-subset share with no events in the window
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06o
mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 --subsets 32 --n 64000 > $O/$tag.json 2>>$O/b.err || { echo "bench $tag failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/$tag.json'));print('$tag',round(a['value']),round(a['ms_per_step'],3))"
}
for R in 1 2; do
  run base_$R MK_NOOP=1
  run mask16_$R MK_LA_MASK=16
  run mask48_$R MK_LA_MASK=48
  run res16_$R MK_RESERVE_CU=16
  run res48_$R MK_RESERVE_CU=48
  run depth1_$R MK_CHOL_DEPTH=1
  run depth3_$R MK_CHOL_DEPTH=3
  run head2_$R MK_LA_HEAD=2
  run head5_$R MK_LA_HEAD=5
  run thr128_$R MK_TILE_THRESH=128
  run thr512_$R MK_TILE_THRESH=512
  run nosplit_$R MK_CHOL_SPLIT=0
done
