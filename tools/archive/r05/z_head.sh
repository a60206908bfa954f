#!/bin/bash
# round 5: MK_LA_HEAD 2 vs 3 at the 32-subset share (interleaved, 4 pairs)
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
for R in 1 2 3 4; do
  for H in 2 3; do
    MK_LA_HEAD=$H timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_h${H}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_h${H}_$R.json'));print('head=$H',round(b['value']))"
  done
done
