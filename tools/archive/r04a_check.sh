#!/bin/bash
# Round 4, first GPU pass after the fault fixes: the GPU suite once (library-default exchange in the
# node tests, watchdog on), the smoke, the 32-subset profiled bench that crashed at exit in round 3,
# then the default bench with its new legs.  Every GPU step has its own time limit; the first failure ends the call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${SUITE_K:+-k "$SUITE_K"} > $O/gpu_tests.log 2>&1 || { echo "suite rc $?"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc $?"; exit 1; }
timeout -k 10 560 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; exit 1; }
tail -c 1500 $O/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof32 -o run -- python3 bench.py --no-cpu-baseline --no-e2e --no-legs --n 64000 --subsets 32 > $O/prof32.log 2>&1
rc=$?; echo "prof32 rc $rc" | tee $O/prof32.rc; exit $rc
