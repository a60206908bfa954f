#!/bin/bash
# round 6 (re-entry): table draws on a side stream -- the kriging tests, then 250 / 32 subsets (40-step windows)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r06zd}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_krig_cheb.py tests/test_gpu_cfg5.py \
  tests/test_gpu_sampler.py tests/test_gpu_node.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 "$@" > $O/$tag.json 2>>$O/b.err || { echo "bench $tag failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/$tag.json'));print('$tag',round(a['value']),round(a['ms_per_step'],3))"
}
for R in 1 2; do
  run b250_$R
  run b32_$R --subsets 32 --n 64000
done
