#!/bin/bash
# round 5: small shards without the split schedule (the fused unsplit factorisation on the lookahead
# candidates' stream) vs the split default -- 32-subset share, configs[1], configs[3] share
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
for R in 1 2; do
  for SP in 1 0; do
    MK_CHOL_SPLIT=$SP timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 --subsets 32 --n 64000 > $O/b32_s${SP}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;b=json.load(open('$O/b32_s${SP}_$R.json'));print('split=$SP 32:',round(b['value']),round(b['ms_per_step'],3))"
  done
done
for SP in 1 0; do
  MK_CHOL_SPLIT=$SP timeout -k 10 240 python bench.py --leg configs1 --steps 40 > $O/c1_s$SP.json 2>>$O/b.err || { echo "leg failed"; tail $O/b.err; exit 1; }
  MK_CHOL_SPLIT=$SP timeout -k 10 240 python bench.py --leg configs3_share7 --steps 40 > $O/s7_s$SP.json 2>>$O/b.err || { echo "leg failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/c1_s$SP.json'));b=json.load(open('$O/s7_s$SP.json'));print('split=$SP configs1', round(a['value'],1), 'share7', round(b['value'],1))"
done
