#!/bin/bash
# round 5: three DMA stages for the diagonal launch's folded correction -- bit identity, then 250 subsets
set -o pipefail
O=gpurun_out/r05f3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_sampler.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2 3; do
  timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  python -c "import json;b=json.load(open('$O/b250_$R.json'));k=b['kernels_ms_per_step'];print('250:',round(b['value']),'diag',round(k['chol_diag'],3),'upd',round(k['chol_update'],3))"
done
