#!/bin/bash
# Round 4: the lean pair sweep as the default; its wave priority (MK_SS_PRIO) beside the GEMM waves
# at 32 subsets, and the masked form (MK_SS_LEAN=0) for reference.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04j}
mkdir -p $O
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
run s32_lean 32
run s32_p1 32 MK_SS_PRIO=1
run s32_p3 32 MK_SS_PRIO=3
run s32_mask 32 MK_SS_LEAN=0
run s32_lean2 32
run s32_p3b 32 MK_SS_PRIO=3
run s250_lean 250
run s250_p3 250 MK_SS_PRIO=3
echo done
