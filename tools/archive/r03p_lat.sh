#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 60 ./tools/diag_probe_np 32 > $O/dp_notasks_32.log 2>&1 || exit 1
