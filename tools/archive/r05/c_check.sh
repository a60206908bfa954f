#!/bin/bash
# round 5: wide kriging GEMM + four-site sweep -- parity, then A/B measurements
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench_kriging.py > $O/krig_wide.json 2> $O/krig.err || { echo krig wide failed; tail $O/krig.err; exit 1; }
MK_PRED_NARROW=1 timeout -k 10 300 python bench_kriging.py --phi-window 0 > $O/krig_narrow.json 2>> $O/krig.err || { echo krig narrow failed; exit 1; }
for f in krig_wide krig_narrow; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',round(d['value']/1e6,2),'M draws/s', d['k_pred_var']['frac'], d['k_pred_var']['avg_launch_ms'], d['cfg5_extrapolation'].get('refreshes_per_kept_sample'), d['cfg5_extrapolation']['seconds_8gpu'])"; done
for Q in 0 1 0 1; do
  MK_SS_QUAD=$Q timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_q$Q.json 2>>$O/b.err || exit 1
  MK_SS_QUAD=$Q timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_q$Q.json 2>>$O/b.err || exit 1
  python -c "import json;a=json.load(open('$O/b250_q$Q.json'));b=json.load(open('$O/b32_q$Q.json'));print('quad=$Q 250:',round(a['value']),round(a['kernels_ms_per_step']['w_sweep'],3),'32:',round(b['value']),round(b['kernels_ms_per_step']['w_sweep'],3))"
done
