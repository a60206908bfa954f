#!/bin/bash
# round 6: event sampling (every 4th iteration) -- bench at 250 and 32 subsets, interleaved with all-launch events
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline_path.py tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for E in 1 4; do
    timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --event-every $E > $O/b250_e${E}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 --event-every $E > $O/b32_e${E}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "
import json;a=json.load(open('$O/b250_e${E}_$R.json'));b=json.load(open('$O/b32_e${E}_$R.json'))
print('every=$E 250:',round(a['value']),round(a['roofline']['frac'],4),a['roofline']['launches'],'32:',round(b['value']),round(b['roofline']['frac'],4),b['roofline']['launches'])"
  done
done
