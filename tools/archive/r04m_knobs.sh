#!/bin/bash
# Round 4: the cooperative multi-workgroup sweep (MK_SWEEP=2) on configs[3]'s 8-GPU share against the
# default split-launch sweep; the lookahead schedule at 250 subsets with the lean sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04m}
mkdir -p $O
leg() {   # name, leg, env...
  local name=$1 l=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --leg $l --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), d.get('kernels_ms_per_step',{}).get('w_sweep'))"
}
leg c3s7_default configs3_share7
leg c3s7_coop configs3_share7 MK_SWEEP=2
leg c3s7_default_b configs3_share7
leg c3s7_coop_b configs3_share7 MK_SWEEP=2
MK_LOOKAHEAD=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --steps 40 > $O/s250_la.json 2> $O/s250_la.err || { echo "s250_la rc $?"; exit 1; }
python -c "import json; d=json.loads(open('$O/s250_la.json').read().strip().splitlines()[-1]); print('s250_la', round(d['value']), round(d['ms_per_step'],3))"
echo done
