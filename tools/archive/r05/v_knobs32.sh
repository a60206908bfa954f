#!/bin/bash
# round 5: the small-shard schedule knobs re-checked on the round-5 build (32 subsets, 40-step windows)
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/$n.json 2>>$O/b.err || { echo "bench $n failed"; tail $O/b.err; exit 1; }
  python -c "import json;b=json.load(open('$O/$n.json'));print('$n',round(b['value']))"
}
for R in 1 2; do
  run default_$R MK_X=0
  run depth1_$R MK_CHOL_DEPTH=1
  run depth3_$R MK_CHOL_DEPTH=3
  run head2_$R MK_LA_HEAD=2
  run head5_$R MK_LA_HEAD=5
  run thresh128_$R MK_TILE_THRESH=128
  run thresh512_$R MK_TILE_THRESH=512
  run reserve48_$R MK_RESERVE_CU=48
done
