#!/bin/bash
# round 5: the GPU suite twice back to back on the final build (stability of the admitted
# multi-workgroup sweep, the fused factorisation and the kriging map under repeated runs)
set -o pipefail
O=gpurun_out/r05st
mkdir -p $O
for R in 1 2; do
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests_$R.log 2>&1 || { echo "suite $R rc $?"; tail -30 $O/gpu_tests_$R.log; exit 1; }
  tail -1 $O/gpu_tests_$R.log
done
