#!/bin/bash
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 120 python tools/r05/krig_diag.py $O/wide.npz || exit 1
MK_PRED_NARROW=1 timeout -k 10 120 python tools/r05/krig_diag.py $O/narrow.npz || exit 1
timeout -k 10 120 python tools/r05/krig_diag.py $O/wide2.npz || exit 1
python - <<'PY'
import numpy as np
a=np.load('gpurun_out/r05d/wide.npz')['pred']; b=np.load('gpurun_out/r05d/narrow.npz')['pred']; c=np.load('gpurun_out/r05d/wide2.npz')['pred']
print('shape', a.shape)
for nm,x in (('wide-narrow',a-b),('wide-wide2',a-c)):
    bad=np.argwhere(np.abs(x)>0)
    print(nm, 'n diff', len(bad), 'max', np.abs(x).max())
    if len(bad): print(bad[:20])
PY
