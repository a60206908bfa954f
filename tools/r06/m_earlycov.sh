#!/bin/bash
# round 6: the sequential schedule's next-iteration covariance assembly beside the sweep (MK_EARLY_COV):
# bit-identity + oracle replays, then 250-subset windows interleaved against MK_EARLY_COV=0
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_headline_path.py tests/test_gpu_sampler.py tests/test_gpu_cfg5.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2 3; do
  for E in 1 0; do
    MK_EARLY_COV=$E timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_e${E}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/b250_e${E}_$R.json'));k=a['kernels_ms_per_step'];print('early=$E 250:',round(a['value']),round(a['ms_per_step'],3),round(a['roofline']['frac'],4),'cov',round(k['cov_candidate'],3),'sweep',round(k['w_sweep'],3))"
  done
done
