#!/bin/bash
# N = 2 bench path rehearsed on one GPU (two gloo ranks share the card).
set -o pipefail
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_2ranks.json 2> gpurun_out/bench_2ranks.err || { tail -8 gpurun_out/bench_2ranks.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_2ranks.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['value'], d['c5_allgather_match'].get('allgather_us'), json.dumps(d['host_input'])[:200], json.dumps(d['device_submit'])[:200])"
