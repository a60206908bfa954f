#!/bin/bash
# round 6: the 32-subset share with the site sweep's workgroups given a CU of their own (LDS reserved
# beyond what a tile-GEMM workgroup can share: MK_SWEEP_LDS_MIN KB), interleaved against the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06e
mkdir -p $O
for R in 1 2; do
  for L in 0 100 128; do
    MK_SWEEP_LDS_MIN=$L timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_l${L}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_l${L}_$R.json'));print('lds_min=$L',round(b['value']),round(b['ms_per_step'],3))"
  done
done
