#!/bin/bash
# round 6: triangular MFMA skips in k_inv_level (phase 0: W_TT's diagonal tile; phase 1: W_BB's) and
# k_pred_var (W_ii) -- full GPU suite, then the 250-subset bench and the kriging leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/b250_$R.json'));print('250:',round(a['value']),round(a['roofline']['frac'],4),'inv',round(a['roofline_inverse']['frac'],4),a['kernels_ms_per_step']['inverse'])"
done
timeout -k 10 300 python bench_kriging.py --phi-window 0 > $O/krig.json 2>>$O/b.err || { echo "krig failed"; tail $O/b.err; exit 1; }
python -c "import json;a=json.load(open('$O/krig.json'));print('krig',round(a['value']/1e6,2),'M/s',round(a['k_pred_var']['frac'],4))"
