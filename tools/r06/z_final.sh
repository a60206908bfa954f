#!/bin/bash
# round 6 final pass on the committed state: GPU suite, smoke, the default bench line, rocprofv3 kernel
# stats of the same command, and the PMC passes for the column-update traffic (bench.py's
# roofline.traffic) and the kriging GEMM
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python - <<PY
import json
b=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=b['roofline']; i=b['roofline_inverse']; L=b['legs']
print('value',round(b['value']),'ms',round(b['ms_per_step'],2),'frac',round(r['frac'],4),r['launches'],round(r['avg_launch_ms'],4),'inv',round(i['frac'],4),'e2e',round(b.get('end_to_end_s',0),1),'cpu',round(b['cpu_baseline']['value'],1))
print('share32',round(L['configs[2]_share32']['value']),'c1',round(L['configs[1]_matern']['value']),'c3',round(L['configs[3]_lmc_share7']['value']),'krig',L['configs[4]_kriging'].get('value'),L['configs[4]_kriging'].get('k_pred_var',{}).get('frac'))
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof250 -o prof -- python3 -u bench.py --no-legs --no-e2e --no-cpu-baseline > $O/prof250.log 2>&1 || { echo "prof failed"; tail -30 $O/prof250.log; exit 1; }
tail -1 $O/prof250.log | cut -c1-200
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  MK_EARLY_COV=0 timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_bench_$lc -- python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-legs --no-e2e > $O/pmc_bench_$lc.log 2>&1 || { echo "pmc bench $c rc $?"; exit 1; }
done
python3 tools/pmc_summary.py $O/pmc_bench_fetch $O/pmc_bench_write $O/pmc_chol_update.json "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-legs --no-e2e"
KR="python3 -u bench_kriging.py --subsets 8 --n-test 262144 --kept 2 --kernel-events 0 --phi-window 0 --fit-chunk 1"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_krig_$lc -- $KR > $O/pmc_krig_$lc.json 2> $O/pmc_krig_$lc.log || { echo "pmc krig $c rc $?"; exit 1; }
done
python3 tools/pmc_summary.py $O/pmc_krig_fetch $O/pmc_krig_write $O/pmc_kriging.json "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- $KR" mk::k_pred_var
