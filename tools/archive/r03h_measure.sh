#!/bin/bash
# Round-3 measurement pass (2/2): per-GPU rate at the strong-scaling shard sizes, end to end configs[0..3].
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h
mkdir -p $O
for K in 32 63 125 188 250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --n $((K * 2000)) --subsets $K >> $O/shard_sizes.jsonl 2>/dev/null || exit 1
done
for c in 1 2 4; do
  timeout -k 10 400 python run_metakriging.py --config $c > $O/e2e_cfg$c.log 2>&1 || exit 1
done
timeout -k 10 400 python run_metakriging.py --config 4 --n 14000 --subsets 7 > $O/e2e_cfg4_share8.log 2>&1 || exit 1
# the multi-GPU bench's node leg (bench.py --e2e-only, what rank 0 starts at N > 1), two blocks on one GPU
timeout -k 10 400 python bench.py --e2e-only --e2e-devices 0,0 > $O/e2e_only_00.json 2> $O/e2e_only_00.err || exit 1
