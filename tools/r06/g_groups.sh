#!/bin/bash
# round 6: the 32-subset share as G concurrent sessions (host threads) on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g
mkdir -p $O
for R in 1 2; do
  for G in 1 2 4; do
    Q=$((G * 8))
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python tools/two_sessions.py --groups $G > $O/g${G}_$R.json 2>>$O/g.err || { echo "run failed"; tail $O/g.err; exit 1; }
    python -c "import json;b=json.load(open('$O/g${G}_$R.json'));print('groups=$G',round(b['value']),round(b['ms_per_step'],3),b['lookahead'],b['sample_checksum'])"
  done
done
