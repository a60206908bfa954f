#!/bin/bash
# round 6: the configs[4] kriging leg at test-site tiles of 65,536 vs 131,072 (fewer repeated kept-state
# factorisations per site; twice the kriging buffers)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06r
mkdir -p $O
for R in 1 2; do
  for T in 65536 131072; do
    timeout -k 10 300 python bench_kriging.py --phi-window 0 --tile $T > $O/krig_t${T}_$R.json 2>>$O/b.err || { echo "krig failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/krig_t${T}_$R.json'));print('tile=$T krig',round(a['value']/1e6,2),'M/s','pred',round(a['predict_seconds'],2),'s',round(a['k_pred_var']['frac'],4))"
  done
done
