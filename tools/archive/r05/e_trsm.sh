#!/bin/bash
# round 5: the two-tile trsm (k_chol_trsm_w) -- bit identity, then A/B at 250 and 32 subsets; the default bench
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_linalg.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for W in 0 1 0 1; do
  MK_TRSM_WIDE=$W timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_w$W.json 2>>$O/b.err || exit 1
  MK_TRSM_WIDE=$W timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_w$W.json 2>>$O/b.err || exit 1
  python -c "import json;a=json.load(open('$O/b250_w$W.json'));b=json.load(open('$O/b32_w$W.json'));print('trsm_wide=$W 250:',round(a['value']),round(a['kernels_ms_per_step']['chol_trsm'],3),'32:',round(b['value']),round(b['kernels_ms_per_step']['chol_trsm'],3))"
done
