#!/bin/bash
# round 5: the sequential schedule's kriging refresh on a side stream beside the sweep -- sampler
# parity, then 250-subset A/B (20- and 40-step windows)
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_linalg.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for K in 1 0; do
    for N in 20 40; do
      MK_SEQ_KRIG=$K timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps $N > $O/b_k${K}_s${N}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
      python -c "import json;a=json.load(open('$O/b_k${K}_s${N}_$R.json'));print('seqkrig=$K steps=$N:',round(a['value']),round(a['ms_per_step'],3))"
    done
  done
done
