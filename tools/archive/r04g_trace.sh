#!/bin/bash
# Round 4: kernel traces of the 32-subset shard, default split schedule vs the chain split.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04g
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-e2e --no-legs --n 64000 --subsets 32 --steps 10"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/def -o run -- $B > $O/def.log 2>&1 || { echo "def rc $?"; exit 1; }
MK_CHOL_CHAIN=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/chain -o run -- $B > $O/chain.log 2>&1 || { echo "chain rc $?"; exit 1; }
echo done
