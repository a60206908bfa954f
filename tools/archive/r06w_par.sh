#!/bin/bash
# round 6 (re-entry): the split Cholesky's off-diagonal correction beside the diagonal launch
# (MK_CHOL_PAR) -- bit-identity test, 32-subset share A/B, one kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_linalg.py \
  -k "bit_identical" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 --subsets 32 --n 64000 > $O/$tag.json 2>>$O/b.err || { echo "bench $tag failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/$tag.json'));print('$tag',round(a['value']),round(a['ms_per_step'],3))"
}
for R in 1 2; do
  run p0_$R MK_CHOL_PAR=0
  run p1_$R MK_CHOL_PAR=1
  run p2_$R MK_CHOL_PAR=2
  run p1d1_$R MK_CHOL_PAR=1 MK_CHOL_DEPTH=1
  run p1d3_$R MK_CHOL_PAR=1 MK_CHOL_DEPTH=3
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr32 -o run -- python3 bench.py --no-legs --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 20 --no-kernel-events > $O/tr32.log 2>&1 || exit 1
python3 tools/stream_timeline.py $O/tr32/run_results.db 305 2 > $O/timeline32_burnin.txt 2>&1 || exit 1
python3 tools/stream_timeline.py $O/tr32/run_results.db 319 2 > $O/timeline32_kept.txt 2>&1 || exit 1
rm -rf $O/tr32
