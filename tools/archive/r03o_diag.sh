#!/bin/bash
# Diagonal-tile probe with per-wave stamps: old pivot (v1), fused-DPP pivot with stores behind the
# pivot chain, fused-DPP pivot with stores at the end.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 60 ./tools/diag_probe_v1 32 > $O/dp_v1_32.log 2>&1 || exit 1
timeout -k 10 60 ./tools/diag_probe 32 > $O/dp_v3_32.log 2>&1 || exit 1
timeout -k 10 60 ./tools/diag_probe_es 32 > $O/dp_v3es_32.log 2>&1 || exit 1
timeout -k 10 60 ./tools/diag_probe 250 > $O/dp_v3_250.log 2>&1 || exit 1
timeout -k 10 60 ./tools/diag_probe_es 250 > $O/dp_v3es_250.log 2>&1 || exit 1
