#!/bin/bash
# round 5: fused update+solve at mid-size shards (the 2-GPU share: 125 subsets, lookahead unsplit; 100 subsets)
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
for R in 1 2; do
  for F in 1 0; do
    for S in 125 100; do
      MK_CHOL_FUSED=$F timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets $S --n $((S*2000)) > $O/b${S}_f${F}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
      python -c "import json;b=json.load(open('$O/b${S}_f${F}_$R.json'));print('fused=$F $S:',round(b['value']),round(b['ms_per_step'],3),b['roofline']['schedule'])"
    done
  done
done
