#!/bin/bash
# round 6 final pass (part c): the PMC passes for the column-update traffic (bench.py's roofline.traffic;
# exact kriging refresh and one adaptation batch, so the serialised run stays short) and the kriging
# GEMM, then a 32-subset kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r06fin}
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  MK_EARLY_COV=0 MK_KRIG_CHEB=0 timeout -s KILL 170 rocprofv3 --pmc $c --output-format csv -d $O/pmc_bench_$lc -- python3 -u bench.py --steps 4 --warmup 1 --adapt-batches 1 --no-cpu-baseline --no-legs --no-e2e > $O/pmc_bench_$lc.log 2>&1 || { echo "pmc bench $c rc $?"; exit 1; }
  echo "pmc bench $c done"
done
python3 tools/pmc_summary.py $O/pmc_bench_fetch $O/pmc_bench_write $O/pmc_chol_update.json "MK_EARLY_COV=0 MK_KRIG_CHEB=0 rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- python3 bench.py --steps 4 --warmup 1 --adapt-batches 1 --no-cpu-baseline --no-legs --no-e2e"
KR="python3 -u bench_kriging.py --subsets 8 --n-test 262144 --kept 2 --kernel-events 0 --phi-window 0 --fit-chunk 1"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 170 rocprofv3 --pmc $c --output-format csv -d $O/pmc_krig_$lc -- $KR > $O/pmc_krig_$lc.json 2> $O/pmc_krig_$lc.log || { echo "pmc krig $c rc $?"; exit 1; }
  echo "pmc krig $c done"
done
python3 tools/pmc_summary.py $O/pmc_krig_fetch $O/pmc_krig_write $O/pmc_kriging.json "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- $KR" mk::k_pred_var
rm -rf $O/pmc_bench_fetch $O/pmc_bench_write $O/pmc_krig_fetch $O/pmc_krig_write
timeout -k 10 170 rocprofv3 --kernel-trace -d $O/tr32 -o run -- python3 bench.py --no-legs --no-cpu-baseline --no-e2e --n 64000 --subsets 32 --steps 20 --no-kernel-events > $O/tr32.json 2> $O/tr32.log || { echo "trace32 failed"; tail $O/tr32.log; exit 1; }
python3 tools/stream_timeline.py $O/tr32/run_results.db 305 2 > $O/timeline32_burnin_305.txt 2>&1 || exit 1
python3 tools/stream_timeline.py $O/tr32/run_results.db 319 2 > $O/timeline32_kept_319.txt 2>&1 || exit 1
python3 tools/db_stats.py $O/tr32/run_results.db > $O/kernel_stats_32.csv 2>&1 || exit 1
rm -rf $O/tr32
head -3 $O/timeline32_burnin_305.txt | cut -c1-200
