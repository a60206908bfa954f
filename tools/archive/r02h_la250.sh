#!/bin/bash
# Lookahead schedule at 250 subsets: rates under mask variants + one kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02h
mkdir -p $O
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 > $O/$lab.json 2> $O/$lab.err || exit 1
}
run seq X=0
run la MK_LOOKAHEAD=1
run la_mask0 MK_LOOKAHEAD=1 MK_LA_MASK=0
run la_krig0 MK_LOOKAHEAD=1 MK_LA_KRIG=0
MK_LOOKAHEAD=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr250 -o run -- python3 bench.py --no-cpu-baseline --no-kernel-events --steps 12 > $O/tr250.log 2>&1 || exit 1
