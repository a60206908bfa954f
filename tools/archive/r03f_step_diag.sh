#!/bin/bash
# After the one-launch-per-block sweep, the 8-way diagonal-tile copy and k_chol_diag's paired stores:
# diag probe, the bit-identity / linalg tests, the sweep variants on configs[3]'s share, 32 / 250 benches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 60 ./tools/diag_probe 32 > $O/diag_probe32.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_sampler.py tests/test_gpu_post.py tests/test_gpu_node.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for K in 7 13; do
  for v in "c4_${K}_step MK_SWEEP=3" "c4_${K}_two MK_SWEEP=4"; do
    set -- $v
    env $2 timeout -k 10 200 python run_metakriging.py --config 4 --n $((K * 2000)) --subsets $K --n-batch 6 > $O/$1.log 2>&1 || exit 1
  done
done
for v in "b32_one MK_SWEEP=1" "b32_step MK_SWEEP=3"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 40 --warmup 4 > $O/$1.json 2> $O/$1.err || exit 1
done
timeout -k 10 150 python bench.py --no-cpu-baseline --no-e2e > $O/b250.json 2> $O/b250.err || exit 1
timeout -k 10 120 ./tools/gemm_probe > $O/gemm_probe.log 2>&1 || exit 1
