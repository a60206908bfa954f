#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/la
mkdir -p $O
B="python bench.py --no-cpu-baseline"
MK_LOOKAHEAD=1 timeout -k 10 200 $B > $O/b250_la1.log 2>&1 || exit 1
MK_LOOKAHEAD=1 MK_LA_MASK=0 timeout -k 10 200 $B > $O/b250_la1_m0.log 2>&1 || exit 1
MK_LOOKAHEAD=1 MK_LA_MASK=16 timeout -k 10 200 $B > $O/b250_la1_m16.log 2>&1 || exit 1
MK_LOOKAHEAD=1 timeout -k 10 200 $B --n 376000 --subsets 188 > $O/b188_la1.log 2>&1 || exit 1
MK_LOOKAHEAD=0 timeout -k 10 200 $B --n 376000 --subsets 188 > $O/b188_la0.log 2>&1 || exit 1
