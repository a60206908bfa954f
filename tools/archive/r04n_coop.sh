#!/bin/bash
# Round 4: the GPU suite twice with the cooperative sweep as the default for q >= 2 small shards (the
# stalls of rounds 2-3 would show here; the watchdog and faulthandler name any), then configs[3]'s
# 8-GPU share window.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n
mkdir -p $O
for r in 1 2; do
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests_$r.log 2>&1 || { echo "suite $r rc $?"; tail -30 $O/gpu_tests_$r.log; exit 1; }
  tail -1 $O/gpu_tests_$r.log
done
timeout -k 10 200 python bench.py --leg configs3_share7 --steps 40 > $O/c3s7.json 2> $O/c3s7.err || { echo "c3s7 rc $?"; exit 1; }
python -c "import json; d=json.loads(open('$O/c3s7.json').read().strip().splitlines()[-1]); print('c3s7', round(d['value']), round(d['ms_per_step'],3))"
echo done
