#!/bin/bash
# round 6: A/B of the triangular MFMA skips (in-tree libmk.so = MK_TRI_SKIP 1; build_ab/libmk_noskip.so = 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06l
mkdir -p $O
NS=$PWD/build_ab/libmk_noskip.so
for R in 1 2 3; do
  for V in skip noskip; do
    L=""; [ $V = noskip ] && L=$NS
    MK_LIB=$L timeout -k 10 200 python bench.py --no-legs --no-e2e --no-cpu-baseline --steps 40 > $O/b250_${V}_$R.json 2>>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/b250_${V}_$R.json'));print('$V 250:',round(a['value']),round(a['roofline']['frac'],4),'inv',round(a['roofline_inverse']['frac'],4),round(a['kernels_ms_per_step']['inverse'],3))"
  done
done
for R in 1 2; do
  for V in skip noskip; do
    L=""; [ $V = noskip ] && L=$NS
    MK_LIB=$L timeout -k 10 300 python bench_kriging.py --phi-window 0 > $O/krig_${V}_$R.json 2>>$O/b.err || { echo "krig failed"; tail $O/b.err; exit 1; }
    python -c "import json;a=json.load(open('$O/krig_${V}_$R.json'));print('$V krig',round(a['value']/1e6,2),'M/s',round(a['k_pred_var']['frac'],4))"
  done
done
