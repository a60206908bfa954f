#!/bin/bash
# round 5: the register-resident trsm (k_chol_trsm_r) -- parity, then A/B at 250 and 32 subsets
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_cfg5.py tests/test_gpu_sampler.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 0 1 0; do
  MK_TRSM_REG=$R timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_r$R.json 2>>$O/b.err || exit 1
  MK_TRSM_REG=$R timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_r$R.json 2>>$O/b.err || exit 1
  python -c "import json;a=json.load(open('$O/b250_r$R.json'));b=json.load(open('$O/b32_r$R.json'));print('trsm_reg=$R 250:',round(a['value']),round(a['kernels_ms_per_step']['chol_trsm'],3),'32:',round(b['value']),round(b['kernels_ms_per_step']['chol_trsm'],3))"
done
