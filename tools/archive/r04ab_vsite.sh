#!/bin/bash
# Round 4: the lean sweep with the sites' data held in registers (v_readlane at a uniform index):
# parity test, then 250- and 32-subset windows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_linalg.py -k "site_sweep" > $O/test_site.log 2>&1 || { echo "site test failed rc $?"; tail -30 $O/test_site.log; exit 1; }
tail -1 $O/test_site.log
run() {   # name, subsets, env...
  local name=$1 S=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((S * 2000)) --subsets $S --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), d['kernels_ms_per_step']['w_sweep'])"
}
run s250 250
run s250_b 250
run s32 32
run s32_b 32
echo done
