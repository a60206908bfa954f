#!/bin/bash
# round 6 (re-entry): the fused table draws in line vs on a side stream (MK_KT_SIDE), 40-step windows
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zh
mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 $EXTRA > $O/$tag.json 2>>$O/b.err || { echo "bench $tag failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/$tag.json'));print('$tag',round(a['value']),round(a['ms_per_step'],3))"
}
for R in 1 2 3; do
  EXTRA="" run b250_s0_$R MK_KT_SIDE=0
  EXTRA="" run b250_s1_$R MK_KT_SIDE=1
  EXTRA="--subsets 32 --n 64000" run b32_s0_$R MK_KT_SIDE=0
  EXTRA="--subsets 32 --n 64000" run b32_s1_$R MK_KT_SIDE=1
done
