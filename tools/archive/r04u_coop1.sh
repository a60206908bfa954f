#!/bin/bash
# Round 4: the cooperative sweep for q = 1 small shards under the lookahead schedule (MK_SWEEP=2)
# against the lean site sweep: 32 subsets and configs[1].
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04u
mkdir -p $O
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
run s32_site 32
run s32_coop 32 MK_SWEEP=2
run s32_site_b 32
run s32_coop_b 32 MK_SWEEP=2
for v in "" 2; do
  MK_SWEEP=$v timeout -k 10 200 python bench.py --leg configs1 --steps 40 > $O/c1_$v.json 2> $O/c1_$v.err || { echo "c1 $v rc $?"; exit 1; }
  python -c "import json; d=json.loads(open('$O/c1_$v.json').read().strip().splitlines()[-1]); print('c1 sweep=$v', round(d['value']), round(d['ms_per_step'],3))"
done
echo done
