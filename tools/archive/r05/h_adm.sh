#!/bin/bash
# round 5: multi-workgroup sweep behind the admission consensus (plain launch, k_sweep fallback) --
# bit identity, the GPU suite's sampler/linalg files, then configs[3]'s 7-subset share A/B vs split launches
set -o pipefail
O=gpurun_out/r05h4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_sampler.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for M in 0 3; do
    MK_SWEEP=$M timeout -k 10 240 python bench.py --leg configs3_share7 --steps 40 > $O/s7_m${M}_$R.json 2>>$O/b.err || { echo "leg failed"; tail $O/b.err; exit 1; }
    python -c "import json;d=json.load(open('$O/s7_m${M}_$R.json'));print('MK_SWEEP=$M run $R', round(d['value'],1), d.get('ms_per_step'), d['schedule'], 'fallbacks', d.get('sweep_fallbacks'))"
  done
done
