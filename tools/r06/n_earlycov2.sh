#!/bin/bash
# round 6: early covariance beside the sweep (1) vs from the decision on (2) vs in-line (0), 250 subsets
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06n
mkdir -p $O
for R in 1 2 3; do
  for E in 1 2 0; do
    MK_EARLY_COV=$E timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_e${E}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/b250_e${E}_$R.json'));k=a['kernels_ms_per_step'];print('early=$E 250:',round(a['value']),round(a['ms_per_step'],3),'cov',round(k['cov_candidate'],3),'sweep',round(k['w_sweep'],3),'inv',round(k['inverse'],3))"
  done
done
MK_EARLY_COV=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_headline_path.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
