#!/bin/bash
# round 5: the lookahead schedule at 250 subsets with the fused factorisation (its diagonal launches
# leave the chip idle on the sequential schedule; lookahead overlaps them with the main stream)
set -o pipefail
O=gpurun_out/r05la
mkdir -p $O
for R in 1 2 3; do
  for L in 1 0; do
    MK_LOOKAHEAD=$L timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_la${L}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b250_la${L}_$R.json'));print('la=$L 250:',round(b['value']),b['roofline']['schedule'])"
  done
done
for L in 1 0; do
  MK_LOOKAHEAD=$L timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 188 --n 376000 > $O/b188_la$L.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  python -c "import json;b=json.load(open('$O/b188_la$L.json'));print('la=$L 188:',round(b['value']),b['roofline']['schedule'])"
done
