#!/bin/bash
# round 6: the default bench line (legs, end to end, CPU baseline) + the N = 2 rehearsal of the rank path
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python - <<PY
import json
b=json.load(open('$O/bench.json'))
r=b['roofline']; i=b['roofline_inverse']; L=b['legs']
print('value',round(b['value']),'ms',round(b['ms_per_step'],2),'frac',round(r['frac'],4),'inv',round(i['frac'],4),'e2e',round(b.get('end_to_end_s',0),1),'cpu',round(b['cpu_baseline']['value'],1))
print('share32',round(L['configs[2]_share32']['value']),'c1',round(L['configs[1]_matern']['value']),'c3',round(L['configs[3]_lmc_share7']['value']),'krig',L['configs[4]_kriging'].get('value'),L['configs[4]_kriging'].get('k_pred_var',{}).get('frac'))
PY
MK_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-cpu-baseline > $O/g2.json 2> $O/g2.err || { echo "gpus 2 failed"; tail -30 $O/g2.err; exit 1; }
python -c "import json;b=json.load(open('$O/g2.json'));print('g2',b['n_gpus'],b['ranks_seen'],b['launcher'],round(b['value']),b['roofline']['launches'])"
