#!/bin/bash
# Round 4: the GPU suite and smoke with the lean pair sweep as the default, then one bench window at
# 250 and at 32 subsets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite rc $?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc $?"; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --steps 40 > $O/s250.json 2> $O/s250.err || { echo "s250 rc $?"; exit 1; }
timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --no-legs --n 64000 --subsets 32 --steps 40 > $O/s32.json 2> $O/s32.err || { echo "s32 rc $?"; exit 1; }
for f in s250 s32; do python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],3), d['kernels_ms_per_step'].get('w_sweep'))"; done
echo done
