#!/bin/bash
# Node driver + tile grids tests, the single-process script over device lists, and the default bench
# (with its measured end-to-end leg).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_sampler.py -k "node or tile_grids or amcmc_length" -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 4 --devices 0 > $O/cfg4_node.log 2>&1 || exit 1
timeout -k 10 200 python run_metakriging.py --config 5 --n 20000 --subsets 10 --n-test 140000 --n-batch 2 --devices 0,0 --combine median > $O/cfg5_node_median.log 2>&1 || exit 1
timeout -k 10 200 python run_metakriging.py --config 5 --n 20000 --subsets 10 --n-test 140000 --n-batch 2 --combine median > $O/cfg5_median.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > $O/bench.log 2> $O/bench.err || exit 1
