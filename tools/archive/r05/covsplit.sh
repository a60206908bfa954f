#!/bin/bash
# round 5: candidate tile columns [c, nt) assembled on a side stream beside the first columns'
# factorisation (MK_COV_SPLIT=c, sequential schedule) -- bit identity, then A/B at 250 subsets
set -o pipefail
O=gpurun_out/r05cs
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for C in 0 2 4 6; do
    MK_COV_SPLIT=$C timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_c${C}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b250_c${C}_$R.json'));k=b['kernels_ms_per_step'];print('covsplit=$C 250:',round(b['value']),round(b['ms_per_step'],3),'frac',round(b['roofline']['frac'],3))"
  done
done
