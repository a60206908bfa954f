#!/bin/bash
# round 6: the MC-error parity tests against 12 independent oracle replicates + the negative control,
# the power probe over perturbed targets, then the sweep-LDS experiment at the 32-subset share
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 300 python -u tools/mc_power.py phi_b:6.5,phi_b:7,iw_s:10 > $O/mc_power.jsonl 2> $O/mc_power.err || { echo "power probe failed"; tail -20 $O/mc_power.err; exit 1; }
python -c "
import json
for l in open('$O/mc_power.jsonl'):
    r=json.loads(l); print(r['case'], r['perturb'], r['criteria_pass'], round(r['max_abs_t_param'],2), round(r['w_frac_gt_3.5'],4), round(r['w_mean_t2'],3))"
timeout -k 10 600 python -u -m pytest tests/test_stat_cfg2_cfg4.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/r06/e_sweeplds.sh
