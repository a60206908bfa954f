#!/bin/bash
# round 6: the cost of the per-launch HIP events in the timed window, at 250 and 32 subsets
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06h
mkdir -p $O
for R in 1 2; do
  for E in "" "--no-kernel-events"; do
    T=$([ -z "$E" ] && echo ev || echo noev)
    timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline $E > $O/b250_${T}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 $E > $O/b32_${T}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/b250_${T}_$R.json'));b=json.load(open('$O/b32_${T}_$R.json'));print('$T 250:',round(a['value']),'32:',round(b['value']))"
  done
done
