#!/bin/bash
# rocprofv3 PMC passes (one counter group per run) for the bench workload and the kriging GEMM.
# Run on the GPU box from the repo root:  bash tools/pmc_passes.sh <tag>
# Writes gpurun_out/pmc_<tag>_{bench,krig}_{fetch,write}/ ; fold with tools/pmc_summary.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=$1
B="python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline"
# the fit one iteration per call (--fit-chunk 1): under --pmc the kernels are serialised and a fit queued in
# one call ran the host far ahead of them -- rocprofiler-sdk's packet intercept then read past the end of a
# mapping (SIGSEGV inside hipLaunchKernel; DESIGN.md 6, profiles/r06/pmc_krig_segv_r05cmd.txt)
KR="python3 -u bench_kriging.py --subsets 8 --n-test 262144 --kept 2 --kernel-events 0 --phi-window 0 --fit-chunk 1"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${T}_bench_$lc -- $B > gpurun_out/pmc_${T}_bench_$lc.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${T}_krig_$lc -- $KR > gpurun_out/pmc_${T}_krig_$lc.log 2>&1
done
