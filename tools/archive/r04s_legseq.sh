#!/bin/bash
# Round 4 diagnostic (pool eviction on): which earlier session still slows a later configs[1] window.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s
mkdir -p $O
for seq in "s32 k c1" "h c1" "h s32 c1"; do
  n=$(echo $seq | tr ' ' '_')
  timeout -k 10 300 python -u tools/leg_seq.py $seq > $O/seq_$n.log 2>&1 || { echo "$seq rc $?"; tail -5 $O/seq_$n.log; exit 1; }
  echo "== $seq"; cat $O/seq_$n.log
done
echo done
