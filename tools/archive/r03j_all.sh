#!/bin/bash
# rows-sweep experiment, then the measurement pass (tests, smoke, default bench, rocprofv3 stats).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/r03i_rows.sh || exit 1
bash tools/r03g_measure.sh || exit 1
