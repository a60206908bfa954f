#!/bin/bash
# round 5: the lookahead kriging stream CU-masked like the main stream (MK_LA_KMASK) -- lookahead
# parity, then A/B at the 32-subset share (3 pairs), configs[1], configs[3]'s share
set -o pipefail
O=gpurun_out/r05km
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2 3; do
  for KM in 1 0; do
    MK_LA_KMASK=$KM timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_k${KM}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_k${KM}_$R.json'));print('kmask=$KM 32:',round(b['value']))"
  done
done
for KM in 1 0; do
  MK_LA_KMASK=$KM timeout -k 10 240 python bench.py --leg configs1 --steps 40 > $O/c1_k$KM.json 2>>$O/b.err || { echo "leg failed"; tail $O/b.err; exit 1; }
  MK_LA_KMASK=$KM timeout -k 10 240 python bench.py --leg configs3_share7 --steps 40 > $O/s7_k$KM.json 2>>$O/b.err || { echo "leg failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/c1_k$KM.json'));b=json.load(open('$O/s7_k$KM.json'));print('kmask=$KM configs1', round(a['value'],1), 'share7', round(b['value'],1))"
done
