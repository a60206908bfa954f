#!/bin/bash
# round 5, first pass: GPU suite (shipped launch pattern: watchdog off), the bench window, and the
# configs[3] 7-subset share under both schedules (split-launch sweep vs cooperative launch)
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python bench.py --no-legs --no-e2e --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['value'],d['roofline']['frac'],d['kernels_ms_per_step'])"
timeout -k 10 200 python bench.py --leg configs3_share7 --steps 40 > $O/c3s7_la.json 2>&1 || exit 1
MK_LOOKAHEAD=0 timeout -k 10 200 python bench.py --leg configs3_share7 --steps 40 > $O/c3s7_seq.json 2>&1 || exit 1
tail -1 $O/c3s7_la.json; tail -1 $O/c3s7_seq.json
