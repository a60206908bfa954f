#!/bin/bash
# Round 4 experiment: several trsm tiles per workgroup (MK_TRSM_REP, MK_TRSM_MINWG): bit-identity on
# the tile-run shards, then 250- and 32-subset windows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04aa
mkdir -p $O
timeout -k 10 200 python tests/gpu_tile_run.py $O/ref.npz > $O/ref.log 2>&1 || { echo "ref rc $?"; exit 1; }
MK_TRSM_REP=4 MK_TRSM_MINWG=1 timeout -k 10 200 python tests/gpu_tile_run.py $O/rep.npz > $O/rep.log 2>&1 || { echo "rep rc $?"; exit 1; }
python -c "
import numpy as np
a=np.load('$O/ref.npz'); b=np.load('$O/rep.npz')
bad=[k for k in a.files if not np.array_equal(a[k], b[k])]
print('bit-identical' if not bad else 'DIFF '+str(bad))
"
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), d['kernels_ms_per_step']['chol_trsm'])"
}
run s250 250
run s250_r2 250 MK_TRSM_REP=2
run s250_r4m512 250 MK_TRSM_REP=4 MK_TRSM_MINWG=512
run s250_r8m256 250 MK_TRSM_REP=8 MK_TRSM_MINWG=256
run s250_b 250
run s32 32
run s32_r4m256 32 MK_TRSM_REP=4 MK_TRSM_MINWG=256
echo done
