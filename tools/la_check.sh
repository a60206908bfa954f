#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/la
mkdir -p $O
if [ "$1" != "notest" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
fi
B="python bench.py --no-cpu-baseline"
S32="--n 64000 --subsets 32"
MK_SWEEP=1 MK_TILE_THRESH=128 timeout -k 10 200 $B $S32 > $O/b32_thr128.log 2>&1 || exit 1
MK_SWEEP=1 MK_TILE_THRESH=192 timeout -k 10 200 $B $S32 > $O/b32_thr192.log 2>&1 || exit 1
MK_TILE_THRESH=256 timeout -k 10 200 $B $S32 > $O/b32_thr256_mg.log 2>&1 || exit 1
MK_LOOKAHEAD=0 MK_TILE_THRESH=256 timeout -k 10 200 $B > $O/b250_thr256_la0.log 2>&1 || exit 1
MK_LOOKAHEAD=1 MK_TILE_THRESH=256 timeout -k 10 200 $B > $O/b250_thr256_la1.log 2>&1 || exit 1
MK_TILE_THRESH=256 timeout -k 10 200 $B --n 250000 --subsets 125 > $O/b125_thr256.log 2>&1 || exit 1
MK_TILE_THRESH=256 MK_SWEEP=1 timeout -k 10 200 $B --n 126000 --subsets 63 > $O/b63_thr256_sw1.log 2>&1 || exit 1
MK_TILE_THRESH=256 timeout -k 10 200 $B --n 126000 --subsets 63 > $O/b63_thr256.log 2>&1 || exit 1
