#!/bin/bash
# round 5: fused update+solve on the split (small-shard) schedule and for small shards -- bit identity
# (linalg + sampler), then the 32-subset share / configs[1] / configs[3] share / 250 A/B
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_sampler.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for F in 1 0; do
    MK_CHOL_FUSED=$F timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_f${F}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_f${F}_$R.json'));k=b['kernels_ms_per_step'];print('fused=$F 32:',round(b['value']),round(b['ms_per_step'],3))"
  done
done
for F in 1 0; do
  MK_CHOL_FUSED=$F timeout -k 10 240 python bench.py --leg configs1 --steps 40 > $O/c1_f$F.json 2>>$O/b.err || { echo "leg failed"; tail $O/b.err; exit 1; }
  MK_CHOL_FUSED=$F timeout -k 10 240 python bench.py --leg configs3_share7 --steps 40 > $O/s7_f$F.json 2>>$O/b.err || { echo "leg failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/c1_f$F.json'));b=json.load(open('$O/s7_f$F.json'));print('fused=$F configs1', round(a['value'],1), 'share7', round(b['value'],1))"
done
MK_CHOL_FUSED=1 timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_f1.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
python -c "import json;b=json.load(open('$O/b250_f1.json'));print('fused=1 250:',round(b['value']),round(b['ms_per_step'],3))"
