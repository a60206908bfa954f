#!/bin/bash
# Round 4: the bench's legs in one process after the stream pool's queue cap (idle streams of other
# kinds evicted before a new queue would exceed GPU_MAX_HW_QUEUES).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04p}
mkdir -p $O
timeout -k 10 400 python bench.py --no-cpu-baseline --no-e2e > $O/bench_legs.json 2> $O/bench_legs.err || { echo "bench rc $?"; tail -5 $O/bench_legs.err; exit 1; }
python - <<PY
import json
d=json.loads(open('$O/bench_legs.json').read().strip().splitlines()[-1])
print('headline', round(d['value']), round(d['ms_per_step'],3))
for k,v in d.get('legs',{}).items(): print(k, round(v['value']), v.get('ms_per_step'))
PY
echo done
