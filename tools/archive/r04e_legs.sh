#!/bin/bash
# Round 4: latent-sweep kernels on configs[1] (Matern, n_s = 1,000) and configs[3] (q = 3), window legs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04e
mkdir -p $O
leg() {   # name, leg, env...
  local name=$1 L=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --leg $L --steps 40 > $O/$name.json 2> $O/$name.err || { echo "$name failed rc $?"; tail -5 $O/$name.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step'],3), d['schedule'])"
}
leg c3s7_site configs3_share7
leg c3s7_step configs3_share7 MK_SWEEP=3
leg c3s7_block configs3_share7 MK_SWEEP=1
leg c1_site configs1
leg c1_pair configs1 MK_SWEEP=7
leg c1_block configs1 MK_SWEEP=1
leg c3_site configs3
leg c3_block configs3 MK_SWEEP=1
