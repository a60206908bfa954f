#!/bin/bash
# round 5: the admitted multi-workgroup sweep at q = 1 (32-subset share, 250 subsets) vs the site sweep
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
for R in 1 2; do
  for M in 0 2; do
    MK_SWEEP=$M timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_m${M}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_m${M}_$R.json'));print('MK_SWEEP=$M 32:',round(b['value']),round(b['kernels_ms_per_step']['w_sweep'],3),round(b['kernels_ms_per_step']['qblocks'],3),'fb',b['sweep_fallbacks'])"
  done
done
MK_SWEEP=2 timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_m2.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
python -c "import json;b=json.load(open('$O/b250_m2.json'));print('MK_SWEEP=2 250:',round(b['value']),round(b['kernels_ms_per_step']['w_sweep'],3),'fb',b['sweep_fallbacks'])"
