#!/bin/bash
# round 6 (re-entry): two subset groups on their own streams at 250 subsets (exact kriging refresh in
# both, the tables need one group), interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zc
mkdir -p $O
run() {  # tag args...
  local tag=$1; shift
  MK_KRIG_CHEB=0 timeout -k 10 300 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 "$@" > $O/$tag.json 2>>$O/b.err || { echo "bench $tag failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/$tag.json'));print('$tag',round(a['value']),round(a['ms_per_step'],3))"
}
for R in 1 2; do
  run g1_$R --streams 1
  run g2_$R --streams 2
done
