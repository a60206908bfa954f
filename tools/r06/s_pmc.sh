#!/bin/bash
# round 6 final PMC passes (one counter group per run): the column-update traffic of the bench command
# (bench.py's roofline.traffic; one adaptation batch so that a serialised pass stays short) and the
# kriging GEMM; then the configs[4] tile-size experiment
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06s
mkdir -p $O
B="python3 -u bench.py --steps 4 --warmup 1 --adapt-batches 1 --no-cpu-baseline --no-legs --no-e2e"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  MK_EARLY_COV=0 timeout -s KILL 170 rocprofv3 --pmc $c --output-format csv -d $O/pmc_bench_$lc -- $B > $O/pmc_bench_$lc.log 2>&1 || { echo "pmc bench $c rc $?"; exit 1; }
  echo "pmc bench $c ok"
done
python3 tools/pmc_summary.py $O/pmc_bench_fetch $O/pmc_bench_write $O/pmc_chol_update.json "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- $B (MK_EARLY_COV=0)"
KR="python3 -u bench_kriging.py --subsets 8 --n-test 262144 --kept 2 --kernel-events 0 --phi-window 0 --fit-chunk 1"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 170 rocprofv3 --pmc $c --output-format csv -d $O/pmc_krig_$lc -- $KR > $O/pmc_krig_$lc.json 2> $O/pmc_krig_$lc.log || { echo "pmc krig $c rc $?"; exit 1; }
  echo "pmc krig $c ok"
done
python3 tools/pmc_summary.py $O/pmc_krig_fetch $O/pmc_krig_write $O/pmc_kriging.json "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- $KR" mk::k_pred_var
bash tools/r06/r_tile.sh
