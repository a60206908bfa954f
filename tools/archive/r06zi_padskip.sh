#!/bin/bash
# round 6 (re-entry): the fused update's padding waves skip their MFMAs -- linalg / sampler / headline-path
# tests, then 250-subset 40-step windows (compare profiles/r06/kside/b250_s1_*)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zi
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_linalg.py tests/test_gpu_sampler.py \
  tests/test_gpu_headline_path.py tests/test_gpu_krig_cheb.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2 3; do
  timeout -k 10 300 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 > $O/b250_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/b250_$R.json'));print('b250_$R',round(a['value']),round(a['ms_per_step'],3))"
done
timeout -k 10 300 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 20 > $O/b250_ev.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
python -c "import json;a=json.load(open('$O/b250_ev.json'));r=a['roofline'];print('b250_ev',round(a['value']),round(r['frac'],4),round(r['avg_launch_ms'],4))"
