#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/la
mkdir -p $O
if [ "$1" != "notest" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
fi
B="python bench.py --no-cpu-baseline"
S32="--n 64000 --subsets 32"
timeout -k 10 200 $B $S32 > $O/b32_mg.log 2>&1 || exit 1
MK_SWEEP_COOP=1 timeout -k 10 200 $B $S32 > $O/b32_mg_coop.log 2>&1 || exit 1
MK_SWEEP=1 timeout -k 10 200 $B $S32 > $O/b32_sweep1.log 2>&1 || exit 1
timeout -k 10 200 $B --n 126000 --subsets 63 > $O/b63.log 2>&1 || exit 1
MK_SWEEP=1 timeout -k 10 200 $B --n 126000 --subsets 63 > $O/b63_sweep1.log 2>&1 || exit 1
MK_LOOKAHEAD=0 timeout -k 10 200 $B --n 126000 --subsets 63 > $O/b63_la0.log 2>&1 || exit 1
