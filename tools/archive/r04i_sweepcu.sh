#!/bin/bash
# Round 4: the lean pair sweep (MK_SS_LEAN: fused-multiply-add dots, no row masks; ring depth 2 via
# MK_SS_H=2) against the shipped form, its parity test, and the sweep on CUs of its own under the
# lookahead schedule (MK_SWEEP_CU, 32 subsets).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_linalg.py -k "site_sweep" > $O/test_site.log 2>&1 || { echo "site test failed rc $?"; tail -30 $O/test_site.log; exit 1; }
tail -3 $O/test_site.log
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
run s32_base 32
run s32_lean 32 MK_SS_LEAN=1
run s32_lean_b 32 MK_SS_LEAN=3
run s32_lean_h2 32 MK_SS_LEAN=1 MK_SS_H=2
run s32_lean_cu32 32 MK_SS_LEAN=1 MK_SWEEP_CU=32
run s32_lean_seq 32 MK_SS_LEAN=1 MK_LOOKAHEAD=0
run s250_base 250
run s250_lean 250 MK_SS_LEAN=1
run s250_lean_h2 250 MK_SS_LEAN=1 MK_SS_H=2
echo done
