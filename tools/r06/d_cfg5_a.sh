#!/bin/bash
# round 6: configs[4]'s per-GPU share end to end, tiles 0..7 (tools/cfg5_share.py; 16 tiles in two calls)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 1100 python -u tools/cfg5_share.py --tiles 0:8 > $O/share_a.json 2> $O/share_a.err || { echo "share a failed rc $?"; tail -20 $O/share_a.err; exit 1; }
tail -3 $O/share_a.err
python -c "import json;r=json.load(open('$O/share_a.json'));print(r['phases_s'],r['x_refreshes_per_kept_sample'])"
