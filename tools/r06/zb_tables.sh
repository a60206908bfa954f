#!/bin/bash
# round 6 (re-entry): fused-path phi tables -- GPU suite, smoke, the full bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r06zb}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python - <<PY
import json
a=json.load(open("$O/bench.json"))
print("value", round(a["value"]), "ms", round(a["ms_per_step"],3), "frac", round(a["roofline"]["frac"],4), "e2e", round(a.get("end_to_end_s") or 0,1))
L=a.get("legs",{})
for k,v in L.items():
    print(k, {kk: v.get(kk) for kk in ("value","ms_per_step") if kk in v}, (v.get("interpolated") or {}).get("cfg5_share_seconds_estimate"))
PY
