#!/bin/bash
# Fused update+trsm Cholesky (MK_CHOL_FUSE, default on): GPU suite, then A/B windows at 32 and 250 subsets.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
for v in "fuse MK_CHOL_FUSE=1" "nofuse MK_CHOL_FUSE=0"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/b32_$1.json 2> $O/b32_$1.err || exit 1
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/b250_$1.json 2> $O/b250_$1.err || exit 1
done
