#!/bin/bash
# Round 4 diagnostic: configs[1] windows after the tiled kriging leg with 1M or 100k sites.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04v
mkdir -p $O
for seq in "c1 k100 c1" "c1 k c1 c1"; do
  n=$(echo $seq | tr ' ' '_')
  timeout -k 10 300 python -u tools/leg_seq.py $seq > $O/seq_$n.log 2>&1 || { echo "$seq rc $?"; tail -5 $O/seq_$n.log; exit 1; }
  echo "== $seq"; cat $O/seq_$n.log
done
echo done
