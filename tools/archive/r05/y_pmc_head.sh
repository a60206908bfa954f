#!/bin/bash
# round 5: kriging PMC passes (k_pred_var bytes per launch after the XCD split; sequential schedule, unsplit:
# under --pmc the small-shard schedules (CU-masked / priority streams) crashed the host process in a
# stream-launch call, rc 139) and MK_LA_HEAD 2 vs 3 at the 32-subset share (interleaved, 4 pairs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05y3
mkdir -p $O
KR="python3 -u bench_kriging.py --subsets 8 --n-test 262144 --kept 2 --kernel-events 0"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  MK_LOOKAHEAD=0 MK_CHOL_SPLIT=0 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc_krig_$lc -- $KR > $O/pmc_krig_$lc.log 2>&1 || { echo "pmc $c rc $?"; exit 1; }
done
for R in 1 2 3 4; do
  for H in 2 3; do
    MK_LA_HEAD=$H timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_h${H}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_h${H}_$R.json'));print('head=$H',round(b['value']))"
  done
done
