#!/bin/bash
# round 5: the lean sweep's W[i, i+1] select -- sampler/linalg parity, then the sweep's cost at 250 / 32 subsets
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_sampler.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/b250_$R.json'));b=json.load(open('$O/b32_$R.json'));print('250:',round(a['value']),round(a['kernels_ms_per_step']['w_sweep'],3),'32:',round(b['value']),round(b['kernels_ms_per_step']['w_sweep'],3))"
done
