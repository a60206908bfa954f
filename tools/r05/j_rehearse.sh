#!/bin/bash
# round 5: rehearse the driver's N-rank bench path on a one-GPU box (bench.py self-launches
# torch.distributed.run; MK_BENCH_REHEARSE puts every rank on GPU 0 over gloo)
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
MK_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-cpu-baseline > $O/g2.json 2> $O/g2.err || { echo "gpus 2 failed"; tail -30 $O/g2.err; exit 1; }
python -c "import json;b=json.load(open('$O/g2.json'));print('g2',b['n_gpus'],b['ranks_seen'],b['launcher'],round(b['value']),b['config']['subsets_per_gpu'])"
MK_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 4 --steps 10 --warmup 2 --no-legs --no-cpu-baseline > $O/g4.json 2> $O/g4.err || { echo "gpus 4 failed"; tail -30 $O/g4.err; exit 1; }
python -c "import json;b=json.load(open('$O/g4.json'));print('g4',b['n_gpus'],b['ranks_seen'],b['launcher'],round(b['value']),b['config']['subsets_per_gpu'])"
