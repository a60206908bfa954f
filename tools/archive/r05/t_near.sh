#!/bin/bash
# round 5: split schedule with the off-diagonal correction on a near stream beside the diagonal launch
# (which folds the diagonal tile's own correction) -- bit identity, then 32-subset / configs[1] A/B
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for NR in 1 0; do
    MK_CHOL_NEAR=$NR timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_n${NR}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_n${NR}_$R.json'));k=b['kernels_ms_per_step'];print('near=$NR 32:',round(b['value']),round(b['ms_per_step'],3))"
  done
done
for NR in 1 0; do
  MK_CHOL_NEAR=$NR timeout -k 10 240 python bench.py --leg configs1 --steps 40 > $O/c1_n$NR.json 2>>$O/b.err || { echo "leg failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/c1_n$NR.json'));print('near=$NR configs1', round(a['value'],1))"
done
