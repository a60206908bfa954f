#!/bin/bash
# Round 4 profiles of the committed defaults: rocprofv3 kernel stats at 250 and 32 subsets, and the
# FETCH_SIZE / WRITE_SIZE passes at 250 (one counter group per run) for the HBM traffic of the
# update kernel and of the site sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04c}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-e2e --no-legs"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof250 -o run -- $B > $O/prof250.log 2>&1 || { echo "prof250 rc $?"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof32 -o run -- $B --n 64000 --subsets 32 > $O/prof32.log 2>&1 || { echo "prof32 rc $?"; exit 1; }
P="python3 -u bench.py --steps 4 --warmup 1 --adapt-batches 0 --no-cpu-baseline --no-e2e --no-legs"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$lc -- $P > $O/pmc_$lc.log 2>&1 || { echo "pmc $c rc $?"; exit 1; }
done
echo done
