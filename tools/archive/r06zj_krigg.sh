#!/bin/bash
# round 6 (re-entry): k_krig_g in 16-column workgroups -- the interpolation tests, 40-step windows at
# 250 / 32 subsets, two tiles of configs[4]'s share (the first makes g)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zj
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_krig_cheb.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 "$@" > $O/$tag.json 2>>$O/b.err || { echo "bench $tag failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/$tag.json'));print('$tag',round(a['value']),round(a['ms_per_step'],3))"
}
for R in 1 2 3; do
  run b250_$R
  run b32_$R --subsets 32 --n 64000
done
timeout -k 10 500 python tools/cfg5_share.py --tiles 0:2 > $O/share_0_2.json 2> $O/share_0_2.err || { echo "share failed"; tail -30 $O/share_0_2.err; exit 1; }
grep "tile" $O/share_0_2.err | tail -2
