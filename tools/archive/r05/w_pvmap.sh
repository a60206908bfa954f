#!/bin/bash
# round 5: k_pred_var's cost-balanced XCD map -- kriging parity (sampler, configs[4] geometry), the
# kriging leg, and the 250-subset bench (kept iterations refresh with uneven pair counts)
set -o pipefail
O=gpurun_out/r05w3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_cfg5.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench_kriging.py > $O/krig.json 2> $O/krig.err || { echo krig failed; tail $O/krig.err; exit 1; }
python -c "import json;d=json.load(open('$O/krig.json'));print('krig',round(d['value']/1e6,2),'M draws/s', d['k_pred_var']['frac'], d['k_pred_var']['avg_launch_ms'], d['cfg5_extrapolation']['seconds_8gpu'])"
for R in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/b250_$R.json'));print('250:',round(a['value']),round(a['ms_per_step'],3))"
done
