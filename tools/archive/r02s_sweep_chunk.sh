#!/bin/bash
# Chunked cooperative multi-workgroup sweep (MK_SWEEP=3) at 250 subsets: bit identity + A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampler.py -m gpu -x -v --timeout 200 --timeout-method thread -k "chunked or sequential" > $O/gpu_tests.log 2>&1 || exit 1
for v in "base X=0" "chunk MK_SWEEP=3" "base2 X=0" "chunk2 MK_SWEEP=3"; do
  set -- $v
  env $2 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 > $O/$1.json 2> $O/$1.err || exit 1
done
