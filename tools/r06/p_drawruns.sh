#!/bin/bash
# round 6: the tiled replay's draws per phi run (MK_DRAW_RUNS) -- parity (tiled == fused, oracle, bit-identity),
# then the configs[4] kriging leg interleaved against per-state draws
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_cfg5.py tests/test_gpu_node.py tests/test_gpu_linalg.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for E in 1 0; do
    MK_DRAW_RUNS=$E timeout -k 10 300 python bench_kriging.py --phi-window 0 > $O/krig_e${E}_$R.json 2>>$O/b.err || { echo "krig failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/krig_e${E}_$R.json'));print('runs=$E krig',round(a['value']/1e6,2),'M/s','pred',round(a['predict_seconds'],2),'s',round(a['k_pred_var']['frac'],4))"
  done
done
