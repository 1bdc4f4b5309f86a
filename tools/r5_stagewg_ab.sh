#!/bin/bash
# Host staging copy kernel size (workgroups) A/B: C++ host loop, micro-batched and not.
set -o pipefail
B=another-cuda-sift_amd/lib/host_pipeline_bench
: > gpurun_out/stagewg_ab.jsonl
for rep in 1 2; do
  for v in sw16 sw24 sw32 sw64; do
    for args in "3 12 300 1 0 4" "3 12 300 2 0 4" "3 6 300 2 0 1"; do
      echo "{\"tag\": \"$v\"}" >> gpurun_out/stagewg_ab.jsonl
      LD_LIBRARY_PATH=ab/L_$v timeout -k 10 120 $B $args >> gpurun_out/stagewg_ab.jsonl 2> gpurun_out/stagewg_ab.err || { tail -5 gpurun_out/stagewg_ab.err; exit 1; }
    done
  done
done
python3 - <<'PY'
import json
tag=None
for l in open('gpurun_out/stagewg_ab.jsonl'):
    l=l.strip()
    if not l.startswith('{'): continue
    d=json.loads(l)
    if 'tag' in d: tag=d['tag']; continue
    print(tag, d['micro_batch'], d['desc'], d['ms_per_frame'])
PY
