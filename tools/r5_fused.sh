#!/bin/bash
# Host results written by the descriptor kernel (HostOut): every GPU test,
# then the pipelined host loop (C++ tool: views / copyToHost / none) and the
# short bench.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/fused_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fused_pytest.log; [ $rc -eq 0 ] || exit 1
B=another-cuda-sift_amd/lib/host_pipeline_bench
: > gpurun_out/fused_host.jsonl
for args in "3 12 300 3 0 4" "3 12 300 1 0 4" "3 12 300 3 0 4" "3 12 300 1 0 4" "3 6 300 3 0 1" "3 6 300 1 0 1" "3 12 300 2 0 4"; do
  timeout -k 10 120 $B $args >> gpurun_out/fused_host.jsonl 2> gpurun_out/fused_host.err || { tail -5 gpurun_out/fused_host.err; exit 1; }
done
grep dev gpurun_out/fused_host.jsonl
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || { tail -5 gpurun_out/bench_fused.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_fused.json').read().strip().splitlines()[-1])
print(d['value'], d['sync_ms_per_frame'], d['exact_descriptors'], json.dumps(d['host_input']), json.dumps(d['device_submit']['micro_batch']))"
