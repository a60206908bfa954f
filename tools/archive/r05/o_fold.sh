#!/bin/bash
# round 5: the diagonal correction folded into k_chol_diag -- bit identity, then A/B at 250 (fold vs
# separate X launch vs unfused) and the mid-size shards (125, 100 subsets: fused vs unfused)
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_sampler.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for F in 1 2 0; do
    MK_CHOL_FUSED=$F timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_f${F}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b250_f${F}_$R.json'));k=b['kernels_ms_per_step'];print('fused=$F 250:',round(b['value']),round(b['ms_per_step'],3),'upd',round(k['chol_update'],3),'sub',round(k['chol_update_sub'],3),'diag',round(k['chol_diag'],3))"
  done
done
for F in 1 0; do
  for S in 125 100; do
    MK_CHOL_FUSED=$F timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets $S --n $((S*2000)) > $O/b${S}_f${F}.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b${S}_f${F}.json'));print('fused=$F $S:',round(b['value']),round(b['ms_per_step'],3),b['roofline']['schedule'])"
  done
done
