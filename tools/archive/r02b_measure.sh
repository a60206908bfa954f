#!/bin/bash
# Round-2 (second session) measurement pass on one MI355X, from the repo root on the GPU box:
# GPU tests, default bench, rocprofv3 kernel stats at 250 and 32 subsets, shard-size sweep,
# end-to-end configs[0..3].
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof32 -o run -- python3 bench.py --no-cpu-baseline --n 64000 --subsets 32 > $O/prof32.log 2>&1 || exit 1
for K in 32 63 125 188 250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --n $((K * 2000)) --subsets $K >> $O/shard_sizes.jsonl 2>/dev/null || exit 1
done
for c in 1 2 3 4; do
  timeout -k 10 400 python run_metakriging.py --config $c > $O/e2e_cfg$c.log 2>&1 || exit 1
done
