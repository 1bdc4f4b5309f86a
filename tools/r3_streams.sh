#!/bin/bash
# Streams x batch sweep (tools/batch_sweep.py), three alternating passes.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/batch_sweep.py --batches ${BATCHES:-16,24,32,48} --streams ${STREAMS:-2,3,4} --frames 1152 > gpurun_out/streams_$r.jsonl 2> gpurun_out/streams_$r.err || { echo "sweep $r failed"; tail -5 gpurun_out/streams_$r.err; exit 1; }
  cat gpurun_out/streams_$r.jsonl
done
