#!/bin/bash
# Round 4 diagnostic: a configs[1] window after the 32-subset shard's session in the same process,
# with the stream pool keeping idle streams (cap 8) or evicting them before a new queue (MK_POOL_CAP).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04q
mkdir -p $O
for cap in 8 5 1; do
  MK_POOL_CAP=$cap timeout -k 10 300 python -u tools/leg_seq.py s32 c1 c3 > $O/seq_cap$cap.log 2>&1 || { echo "cap $cap rc $?"; tail -5 $O/seq_cap$cap.log; exit 1; }
  echo "cap $cap"; cat $O/seq_cap$cap.log
done
echo done
