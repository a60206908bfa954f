#!/bin/bash
# Round 4: the GEMM tile policy at the 32-subset share now that its iteration is bound by total work
# (MK_TILE_THRESH: 128-tiles for launches of at least that many 128-tile workgroups, default 256).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04z
mkdir -p $O
run() {   # name, env...
  local name=$1; shift 1
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n 64000 --subsets 32 --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
run def
run t128 MK_TILE_THRESH=128
run t64 MK_TILE_THRESH=64
run t1 MK_TILE_THRESH=1
run def_b
run t128_b MK_TILE_THRESH=128
echo done
