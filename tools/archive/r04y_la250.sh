#!/bin/bash
# Round 4: the lookahead schedule at 250 subsets (MK_LOOKAHEAD=1) against the default sequential one,
# three 40-step windows each, interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04y
mkdir -p $O
run() {   # name, env...
  local name=$1; shift 1
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3))"
}
for r in 1 2 3; do
  run seq_$r
  run la_$r MK_LOOKAHEAD=1
done
echo done
