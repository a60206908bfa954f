#!/bin/bash
# Round 5 pass on the committed defaults: GPU suite, smoke, the default bench (all legs, CPU baseline,
# end to end), rocprofv3 kernel stats at 250 and 32 subsets, FETCH_SIZE / WRITE_SIZE passes at 250.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r05g}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite rc $?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc $?"; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'e2e', round(d.get('end_to_end_s',0),1), 'cpu', round(d['cpu_baseline']['value'],1), 'legs', {k: round(v.get('value',0)) for k,v in d.get('legs',{}).items()})"
B="python3 bench.py --no-cpu-baseline --no-e2e --no-legs"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof250 -o run -- $B > $O/prof250.log 2>&1 || { echo "prof250 rc $?"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof32 -o run -- $B --n 64000 --subsets 32 > $O/prof32.log 2>&1 || { echo "prof32 rc $?"; exit 1; }
P="python3 -u bench.py --steps 4 --warmup 1 --adapt-batches 0 --no-cpu-baseline --no-e2e --no-legs"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$lc -- $P > $O/pmc_$lc.log 2>&1 || { echo "pmc $c rc $?"; exit 1; }
done
echo done
