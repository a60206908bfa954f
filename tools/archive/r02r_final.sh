#!/bin/bash
# Round-2 re-entry final measurement pass on one MI355X: default bench (with the CPU baseline),
# shard-size sweep, end-to-end configs[0..3], 1M-site kriging sample.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit 1
for K in 32 63 125 188 250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --n $((K * 2000)) --subsets $K >> $O/shard_sizes.jsonl 2>/dev/null || exit 1
done
for c in 1 2 3 4; do
  timeout -k 10 400 python run_metakriging.py --config $c > $O/e2e_cfg$c.log 2>&1 || exit 1
done
timeout -k 10 300 python bench_kriging.py > $O/kriging_1M.json 2> $O/kriging_1M.err || exit 1
