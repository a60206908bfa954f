#!/bin/bash
# round 6 (re-entry): BASELINE configs[4] as one job on ONE GPU -- n = 500k, K = 250 subsets of 2,000,
# 100 x 50 amcmc iterations (1,251 kept), spPredict of 1,000,000 held-out sites through the
# phi-interpolated tiled replay, the combine tile by tile, MK.R:136-165's summary
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zl
mkdir -p $O
timeout -k 10 1120 python -u run_metakriging.py --config 5 > $O/cfg5_full.json 2> $O/cfg5_full.err || { echo "cfg5 failed rc $?"; tail -20 $O/cfg5_full.err; exit 1; }
tail -3 $O/cfg5_full.err
python -c "import json;a=json.load(open('$O/cfg5_full.json'));print(a['phases'], a.get('param_median'), a.get('w_test_coverage_95'))"
