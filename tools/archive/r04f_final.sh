#!/bin/bash
# Round 4 pass on the chosen defaults: suite, smoke, the default bench (all legs, CPU baseline, end to
# end), rocprofv3 kernel stats at 250 and 32 subsets, FETCH / WRITE passes at 250.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04f}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite rc $?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc $?"; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'e2e', round(d.get('end_to_end_s',0),1), 'cpu', round(d['cpu_baseline']['value'],1))"
O=$O bash tools/r04c_prof.sh
