#!/bin/bash
# Kriging GEMM raster (MK_PRED_GI) A/B at configs[4] scale + kernel stats of the tiled kriging.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_linalg.py -m gpu -x -v --timeout 280 --timeout-method thread -k bit_identical > $O/gpu_tests.log 2>&1 || exit 1
for gi in 1 4 8 2; do
  MK_PRED_GI=$gi timeout -k 10 200 python bench_kriging.py > $O/krig_gi$gi.json 2> $O/krig_gi$gi.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profk -o run -- python3 bench_kriging.py --kernel-events 0 > $O/profk.log 2>&1 || exit 1
