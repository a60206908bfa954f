#!/bin/bash
# Round 5 closing pass: the evidence recipe (suite, smoke, default bench, rocprofv3 stats, PMC passes)
# then the one-GPU rehearsal of the N-rank bench path
set -o pipefail
O=${O:-gpurun_out/r05u}
O=$O bash tools/r05/l_final.sh || exit 1
MK_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-cpu-baseline > $O/g2.json 2> $O/g2.err || { echo "gpus 2 failed"; tail -30 $O/g2.err; exit 1; }
python -c "import json;b=json.load(open('$O/g2.json'));print('rehearsal g2',b['n_gpus'],b['ranks_seen'],round(b['value']))"
