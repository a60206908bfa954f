#!/bin/bash
# Kriging raster (MK_PRED_GI) at the configs[2] shape (n_test = 1,000: 8 test tiles per pair).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02p
mkdir -p $O
for gi in 1 8 4 16 1; do
  MK_PRED_GI=$gi timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 > $O/gi$gi.json 2> $O/gi$gi.err || exit 1
  python - "$O/gi$gi.json" >> $O/summary.txt <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); print(sys.argv[1], d["value"], d["ms_per_step"], d["kernels_ms_per_step"])
PY
done
