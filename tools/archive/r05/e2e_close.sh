#!/bin/bash
# Round 5 closing: shard-size rates (configs[2]'s subsets, 40-step windows) and end to end configs[0],
# [1], [3] and [3]'s 8-GPU share through run_metakriging.py (the reference script's whole flow)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05e2e
mkdir -p $O
for K in 32 63 125 188 250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-legs --steps 40 --n $((K * 2000)) --subsets $K >> $O/shard_sizes.jsonl 2>>$O/b.err || { echo "shard $K failed"; exit 1; }
  tail -1 $O/shard_sizes.jsonl | python -c "import json,sys;b=json.loads(sys.stdin.read());print('shard $K', round(b['value']))"
done
for c in 1 2 4; do
  timeout -k 10 400 python run_metakriging.py --config $c > $O/e2e_cfg$c.log 2>&1 || { echo "e2e $c failed"; tail $O/e2e_cfg$c.log; exit 1; }
  grep -i "end.to.end\|wall" $O/e2e_cfg$c.log | tail -2
done
timeout -k 10 400 python run_metakriging.py --config 4 --n 14000 --subsets 7 > $O/e2e_cfg4_share8.log 2>&1 || { echo "e2e share failed"; exit 1; }
grep -i "end.to.end\|wall" $O/e2e_cfg4_share8.log | tail -2
