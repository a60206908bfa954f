#!/bin/bash
# round 6 final pass (part a) on the committed state: GPU suite, smoke, the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r06fin}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python - <<PY
import json
b=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=b['roofline']; i=b['roofline_inverse']; L=b['legs']
print('value',round(b['value']),'ms',round(b['ms_per_step'],2),'frac',round(r['frac'],4),r['launches'],round(r['avg_launch_ms'],4),'inv',round(i['frac'],4),'e2e',round(b.get('end_to_end_s',0),1),'cpu',round(b['cpu_baseline']['value'],1), 'x', round(b['gpu_over_cpu'],1))
k=L['configs[4]_kriging']
print('share32',round(L['configs[2]_share32']['value']),'c1',round(L['configs[1]_matern']['value']),'c3',round(L['configs[3]_lmc_share7']['value']),'krig',k.get('value'),k.get('k_pred_var',{}).get('frac'), k.get('interpolated',{}).get('cfg5_share_seconds_estimate'), k.get('interpolated',{}).get('draws_per_s'))
PY
timeout -k 10 600 python tools/cfg5_share.py --tiles 0:16 > $O/share_0_16.json 2> $O/share_0_16.err || { echo "share failed"; tail -20 $O/share_0_16.err; exit 1; }
python -c "import json;a=json.load(open('$O/share_0_16.json'));p=a['phases_s'];print('cfg5 share', round(p['chains_s']+p['param_grids_s']+p['tiles_replay_grids_s']+p['tiles_combine_s'],1), a['interpolated_tiles'], a['fallback_tiles'], a['max_check_difference'], a['exact_evaluations'])"
