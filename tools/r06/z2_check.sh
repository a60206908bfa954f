#!/bin/bash
# round 6 (re-entry): GPU suite, smoke, the kriging bench child (6-state exact sample + the
# interpolated share's first two tiles) and configs[4]'s whole per-GPU share (phi-interpolated)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r06z2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python bench_kriging.py > $O/krig.json 2> $O/krig.err || { echo "krig failed"; tail -20 $O/krig.err; exit 1; }
python -c "import json;a=json.load(open('$O/krig.json'));print(round(a['value']/1e6,2),'M draws/s exact sample', a['k_pred_var']['frac']);print(a['interpolated'])"
timeout -k 10 900 python tools/cfg5_share.py --tiles 0:16 > $O/share_0_16.json 2> $O/share_0_16.err || { echo "share failed"; tail -20 $O/share_0_16.err; exit 1; }
python -c "import json;a=json.load(open('$O/share_0_16.json'));print(a['phases_s'], a['interpolated_tiles'], a['fallback_tiles'], a['max_check_difference'])"
