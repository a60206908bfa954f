#!/bin/bash
# round 5: the wide kriging GEMM (k_pred_var_w) -- parity first, then the configs[4] leg A/B
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cfg5.py tests/test_gpu_linalg.py tests/test_gpu_sampler.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench_kriging.py > $O/krig_wide.json 2> $O/krig_wide.err || { echo krig wide failed; tail $O/krig_wide.err; exit 1; }
MK_PRED_NARROW=1 timeout -k 10 300 python bench_kriging.py > $O/krig_narrow.json 2> $O/krig_narrow.err || { echo krig narrow failed; exit 1; }
timeout -k 10 300 python bench_kriging.py > $O/krig_wide2.json 2>> $O/krig_wide.err || exit 1
for f in krig_wide krig_narrow krig_wide2; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',round(d['value']/1e6,2),'M draws/s', d['k_pred_var']['frac'], d['k_pred_var']['avg_launch_ms'])"; done
