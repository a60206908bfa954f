#!/bin/bash
# Round 4 experiment: the site sweep requesting a whole CU's LDS (MK_SS_FULLCU, KB) so that no GEMM
# workgroup shares its CU under the lookahead schedule (32 subsets).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04w
mkdir -p $O
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
run s32 32
run s32_full100 32 MK_SS_FULLCU=100
run s32_full150 32 MK_SS_FULLCU=150
run s32_b 32
run s32_full100_b 32 MK_SS_FULLCU=100
echo done
