#!/bin/bash
# round 6: the clock the chip holds under the fp64 GEMM load (GRBM_GUI_ACTIVE / 8 / kernel time) and
# where the column-update waves spend their cycles (SQ wave-state counters); one counter group per run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
grep -E "GRBM_GUI_ACTIVE|GRBM_COUNT|SQ_WAVE_CYCLES|SQ_WAIT_ANY|SQ_WAIT_INST_ANY|SQ_ACTIVE_INST_ANY|SQ_VALU_MFMA_BUSY_CYCLES|SQ_BUSY_CYCLES|SQ_INSTS_VALU_MFMA_MOPS_F64" $O/counters_list.txt | head -20 || true
B="python3 -u bench.py --steps 4 --warmup 1 --adapt-batches 1 --no-cpu-baseline --no-legs --no-e2e"
MK_EARLY_COV=0 timeout -s KILL 170 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/pmc_grbm -- $B > $O/pmc_grbm.log 2>&1 || { echo "grbm rc $?"; exit 1; }
echo "grbm ok"
MK_EARLY_COV=0 timeout -s KILL 170 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -- $B > $O/pmc_sq.log 2>&1 || { echo "sq rc $?"; exit 1; }
echo "sq ok"
