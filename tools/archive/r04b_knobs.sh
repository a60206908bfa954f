#!/bin/bash
# Round 4: the site sweep and the chain-split Cholesky against the round-3 defaults, one bench window
# each (no CPU baseline, no end-to-end, no legs): 32 subsets (the 8-GPU share) and 250.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04b}
mkdir -p $O
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
run s32_site 32
run s32_block 32 MK_SWEEP=1
run s32_pair 32 MK_SWEEP=7
run s32_chain1 32 MK_CHOL_CHAIN=1
run s32_chain2 32 MK_CHOL_CHAIN=2
run s32_fuse 32 MK_COV_FUSE=1
run s250_site 250
run s250_fuse 250 MK_COV_FUSE=1
run s250_block 250 MK_SWEEP=1
run s250_pair 250 MK_SWEEP=7
