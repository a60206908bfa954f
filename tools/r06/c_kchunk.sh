#!/bin/bash
# round 6: the split Cholesky's bulk update in K-chunks (MK_BULK_KCHUNK) -- bit-identity, then the
# 32-subset share (the per-GPU work of an 8-GPU run) interleaved against the unchunked default;
# then (last: it may end in a host SIGSEGV) the kriging PMC passes, tools/r06/b_pmc_krig.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py -k "bit_identical" -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for C in 0 1 2 4; do
    MK_BULK_KCHUNK=$C timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_c${C}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_c${C}_$R.json'));print('kchunk=$C',round(b['value']),round(b['ms_per_step'],3))"
  done
done
bash tools/r06/b_pmc_krig.sh
