#!/bin/bash
# round 6: the site sweep's waves at issue priority 3 (build_ab/libmk_prio3.so) beside the early covariance
# assembly, 250 subsets, interleaved against the in-tree build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06v
mkdir -p $O
PL=$PWD/build_ab/libmk_prio3.so
for R in 1 2 3; do
  for V in base prio; do
    L=""; [ $V = prio ] && L=$PL
    MK_LIB=$L timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_${V}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/b250_${V}_$R.json'));k=a['kernels_ms_per_step'];print('$V 250:',round(a['value']),round(a['ms_per_step'],3),'cov',round(k['cov_candidate'],3),'sweep',round(k['w_sweep'],3))"
  done
done
for R in 1 2; do
  for V in base prio; do
    L=""; [ $V = prio ] && L=$PL
    MK_LIB=$L timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 --subsets 32 --n 64000 > $O/b32_${V}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/b32_${V}_$R.json'));print('$V 32:',round(a['value']),round(a['ms_per_step'],3))"
  done
done
