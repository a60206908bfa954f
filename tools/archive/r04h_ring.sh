#!/bin/bash
# Round 4: the site sweep's W ring depth (MK_SS_H columns per half; default 4) at 32 and 250 subsets,
# and the sweep alone at 32 subsets (sequential schedule).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04h}
mkdir -p $O
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
run s32_h4 32
run s32_h2 32 MK_SS_H=2
run s32_h6 32 MK_SS_H=6
run s32_h8 32 MK_SS_H=8
run s32_fma 32 MK_SS_H=100
run s32_fma8 32 MK_SS_H=108
run s32_seq_h4 32 MK_LOOKAHEAD=0
run s32_seq_h8 32 MK_LOOKAHEAD=0 MK_SS_H=8
run s32_res48 32 MK_RESERVE_CU=48 MK_LA_MASK=48
run s32_res64 32 MK_RESERVE_CU=64 MK_LA_MASK=64
run s32_res64m32 32 MK_RESERVE_CU=64
run s250_h4 250
run s250_h2 250 MK_SS_H=2
run s250_h6 250 MK_SS_H=6
run s250_h8 250 MK_SS_H=8
run s250_fma 250 MK_SS_H=100
run s250_fma8 250 MK_SS_H=108
echo done
