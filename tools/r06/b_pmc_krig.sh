#!/bin/bash
# round 6: the kriging leg's PMC passes with the fit run one iteration per mk_session_run call (the
# device idle after each) -- r06a's SIGSEGV diagnostic put the fault in rocprofiler-sdk's packet
# intercept under a launch call while the host ran iterations ahead of the serialised kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06b
mkdir -p $O
KR="python3 -u bench_kriging.py --subsets 8 --n-test 262144 --kept 2 --kernel-events 0 --phi-window 0 --fit-chunk 1"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  MK_SEGV_DIAG=$PWD/$O/segv_$lc.txt timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_krig_$lc -- $KR > $O/pmc_krig_$lc.json 2> $O/pmc_krig_$lc.log || { echo "pmc $c rc $?"; grep -v "^    @" $O/pmc_krig_$lc.log | tail -5; exit 1; }
  echo "pmc $c ok"
done
python3 tools/pmc_summary.py $O/pmc_krig_fetch $O/pmc_krig_write $O/pmc_kriging.json "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- $KR" mk::k_pred_var
