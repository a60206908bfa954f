#!/bin/bash
# configs[3] 8-GPU share (7 subsets, q = 3): cooperative-launched multi-workgroup sweep under lookahead.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02z
mkdir -p $O
for v in "base X=0" "coop MK_SWEEP=2,MK_SWEEP_COOP=1" "plain MK_SWEEP=2"; do
  set -- $v
  env ${2//,/ } timeout -k 10 120 python run_metakriging.py --config 4 --n 14000 --subsets 7 --n-batch 6 > $O/$1.log 2>&1 || exit 1
done
timeout -k 10 150 python bench.py --no-cpu-baseline --n 64000 --subsets 32 --steps 20 > $O/b32.json 2> $O/b32.err || exit 1
