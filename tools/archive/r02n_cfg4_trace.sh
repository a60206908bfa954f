#!/bin/bash
# Short kernel trace of configs[3] (q = 3 LMC, 50 subsets of 2000) and the 32-subset bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02n
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/cfg4 -o run -- python3 run_metakriging.py --config 4 --n-batch 1 --batch-length 40 > $O/cfg4.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32.json 2> $O/b32.err || exit 1
