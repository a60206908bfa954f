#!/bin/bash
# Round 4 close: end-to-end configs[0], [1], [3] (and [3]'s 8-GPU share) and shard-size rates with
# the round-4 defaults (lean sweep, cooperative q >= 2 small-shard sweep, pool eviction).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ad
mkdir -p $O
for c in 1 2 4; do
  timeout -k 10 400 python run_metakriging.py --config $c > $O/e2e_cfg$c.log 2>&1 || { echo "cfg$c rc $?"; tail -5 $O/e2e_cfg$c.log; exit 1; }
  echo "cfg$c"; grep -i "wall\|seconds\|elapsed\|total" $O/e2e_cfg$c.log | tail -3
done
timeout -k 10 400 python run_metakriging.py --config 4 --n 14000 --subsets 7 > $O/e2e_cfg4_share8.log 2>&1 || { echo "share8 rc $?"; exit 1; }
echo "cfg4 share8"; grep -i "wall\|seconds\|elapsed\|total" $O/e2e_cfg4_share8.log | tail -3
for K in 32 63 125 188 250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-legs --n $((K * 2000)) --subsets $K --steps 40 >> $O/shard_sizes.jsonl 2>/dev/null || { echo "K=$K rc $?"; exit 1; }
done
python -c "
import json
for l in open('$O/shard_sizes.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d['config']['subsets_per_gpu'], round(d['value']), round(d['ms_per_step'],3))
"
echo done
