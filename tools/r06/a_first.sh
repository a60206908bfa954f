#!/bin/bash
# round 6, first GPU pass: the headline-path oracle test + linalg parity, the bench with the
# algorithmic roofline and the inverse's fraction, rocprofv3 stats of the same command, and (last,
# since it may end in a host SIGSEGV) the kriging PMC pass with the SIGSEGV diagnostic installed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline_path.py tests/test_gpu_linalg.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --no-legs --no-e2e --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python -c "import json;b=json.load(open('$O/bench.json'));r=b['roofline'];i=b['roofline_inverse'];print('value',round(b['value']),'frac',round(r['frac'],4),'avg',round(r['avg_launch_ms'],4),'GF/l',r['algorithmic_flops_per_launch']/1e9,'inv',round(i['frac'],4),i['avg_launch_ms'],i['launches'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof250 -o prof -- python3 -u bench.py --no-legs --no-e2e --no-cpu-baseline > $O/prof250.log 2>&1 || { echo "prof failed"; tail -30 $O/prof250.log; exit 1; }
tail -1 $O/prof250.log | cut -c1-300
MK_SEGV_DIAG=$PWD/$O/segv.txt timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_krig_fetch -- python3 -u bench_kriging.py --subsets 8 --n-test 262144 --kept 2 --kernel-events 0 > $O/pmc_krig_fetch.log 2>&1
echo "pmc krig rc $?"
ls -la $O
