#!/bin/bash
# round 5: 64-row parts for the late fused launches at 250 subsets (MK_TILE_THRESH), 2 pairs
set -o pipefail
O=gpurun_out/r05th
mkdir -p $O
for R in 1 2; do
  for T in 256 1024 2048; do
    MK_TILE_THRESH=$T timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_t${T}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b250_t${T}_$R.json'));k=b['kernels_ms_per_step'];print('thresh=$T 250:',round(b['value']),'upd',round(k['chol_update'],3),'sub',round(k['chol_update_sub'],3),'inv',round(k['inverse'],3))"
  done
done
