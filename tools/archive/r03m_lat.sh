#!/bin/bash
# Latency fixes in the per-subset kernels (batched loads in k_beta / k_Aphase / k_trmv_Z, LDS-DMA
# Q_BB and batched partials in k_sweep_step): GPU suite, then configs[3]'s 8-GPU share and the
# 32-subset shard.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${R03M_OUT:-r03m}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python run_metakriging.py --config 4 --n 14000 --subsets 7 > $O/cfg4_share8.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32.json 2> $O/b32.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/q3step -o run -- python3 run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 6 > $O/q3step.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/b250.json 2> $O/b250.err || exit 1
