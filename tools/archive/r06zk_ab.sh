#!/bin/bash
# round 6 (re-entry): interleaved A/B at 250 subsets (40-step windows) of the in-tree library against
# two variants built with compile-time switches (tools/libmk_*.so): MK_KRIGG_COLS=1 (one-column k_krig_g
# workgroups) and MK_PADSKIP=1 (the fused update's all-padding waves skip their MFMAs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zk
mkdir -p $O
timeout -k 10 300 env MK_LIB=$PWD/tools/libmk_pad.so python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_linalg.py > $O/tests_pad.log 2>&1 || { echo "pad tests failed"; tail -30 $O/tests_pad.log; exit 1; }
tail -1 $O/tests_pad.log
run() {  # tag lib
  local tag=$1; local lib=$2
  env ${lib:+MK_LIB=$lib} timeout -k 10 300 python bench.py --no-legs --no-e2e --no-cpu-baseline --no-kernel-events --steps 40 > $O/$tag.json 2>>$O/b.err || { echo "bench $tag failed"; tail $O/b.err; exit 1; }
  python -c "import json;a=json.load(open('$O/$tag.json'));print('$tag',round(a['value']),round(a['ms_per_step'],3))"
}
for R in 1 2 3; do
  run base_$R ""
  run k1_$R $PWD/tools/libmk_k1.so
  run pad_$R $PWD/tools/libmk_pad.so
done
