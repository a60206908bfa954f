#!/bin/bash
# Round 4: the sweep on a high-priority stream under the lookahead schedule (MK_SWEEP_HP), 32 subsets;
# and configs[1] / configs[3]-share windows with the lean sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04k}
mkdir -p $O
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
run s32_lean 32
run s32_hp 32 MK_SWEEP_HP=1
run s32_lean_b 32
run s32_hp_b 32 MK_SWEEP_HP=1
run s63_lean 63
run s63_hp 63 MK_SWEEP_HP=1
for leg in configs1 configs3_share7; do
  timeout -k 10 200 python bench.py --leg $leg --steps 40 > $O/$leg.json 2> $O/$leg.err || { echo "$leg failed rc $?"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$leg.json').read().strip().splitlines()[-1]); print('$leg', {k: d[k] for k in d if k in ('value','ms_per_step')})"
done
echo done
