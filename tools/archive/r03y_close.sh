#!/bin/bash
# Closing checks: the GPU suite with RCCL kept out of the test process, shard-size rates and
# end-to-end configs[0], [1], [3] (and [3]'s 8-GPU share) after the diagonal-tile rework.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v > $O/gpu_tests.log 2>&1 || exit 1
for K in 32 63 125 188 250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --n $((K * 2000)) --subsets $K >> $O/shard_sizes.jsonl 2>/dev/null || exit 1
done
for c in 1 2 4; do
  timeout -k 10 400 python run_metakriging.py --config $c > $O/e2e_cfg$c.log 2>&1 || exit 1
done
timeout -k 10 400 python run_metakriging.py --config 4 --n 14000 --subsets 7 > $O/e2e_cfg4_share8.log 2>&1 || exit 1
