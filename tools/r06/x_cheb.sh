#!/bin/bash
# round 6 (re-entry): phi-interpolated tiled kriging -- its tests, the tiled path's tests, and two
# tiles of configs[4]'s per-GPU share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r06x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_krig_cheb.py \
  tests/test_gpu_cfg5.py "tests/test_gpu_sampler.py::test_tiled_kriging_is_bit_identical_to_fused" \
  "tests/test_gpu_node.py::test_session_tile_grids_equal_the_whole_grids" > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 500 python tools/cfg5_share.py --tiles 0:2 > $O/share_0_2.json 2> $O/share_0_2.err || { echo "share failed"; tail -30 $O/share_0_2.err; exit 1; }
tail -5 $O/share_0_2.err
python -c "import json;a=json.load(open('$O/share_0_2.json'));print({k:a[k] for k in ('phases_s','per_tile','interpolated_tiles','exact_evaluations','max_check_difference','fallback_tiles','x_refreshes_per_kept_sample')})"
