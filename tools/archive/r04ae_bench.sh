#!/bin/bash
# Round 4: the default bench with the configs[4] kriging leg in a child process.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; tail -5 $O/bench.err; exit 1; }
python - <<PY
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', round(d['value']), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'cpu', round(d['cpu_baseline']['value'],1))
for k,v in d['legs'].items(): print(k, v.get('value'), v.get('process'), v.get('error'), (v.get('k_pred_var') or {}).get('frac'))
PY
