#!/bin/bash
# round 5: W's diagonal-tile copy folded into the first inverse level -- linalg/sampler parity, then
# 32- and 250-subset windows
set -o pipefail
O=gpurun_out/r05cf
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_sampler.py tests/test_gpu_cfg5.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2 3; do
  timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/b32_$R.json'));b=json.load(open('$O/b250_$R.json'));print('32:',round(a['value']),'250:',round(b['value']),'inv',round(b['kernels_ms_per_step']['inverse'],3))"
done
