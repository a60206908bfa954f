#!/bin/bash
# Round-2 measurement pass on one MI355X (run from the repo root on the GPU box).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof250 -o run -- python3 bench.py --no-cpu-baseline > $O/prof250.log 2>&1
MK_SWEEP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof32 -o run -- python3 bench.py --no-cpu-baseline --n 64000 --subsets 32 > $O/prof32.log 2>&1
for K in 32 63 125 250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --n $((K * 2000)) --subsets $K >> $O/shard_sizes.jsonl 2>/dev/null
done
for c in 1 2 3 4; do
  timeout -k 10 400 python run_metakriging.py --config $c > $O/e2e_cfg$c.log 2>&1
done
