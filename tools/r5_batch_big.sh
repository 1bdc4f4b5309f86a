#!/bin/bash
# Larger frame batches for the headline leg: B = 16, 24, 32 at 2 and 3 streams.
set -o pipefail
timeout -k 10 500 python tools/batch_sweep.py --batches 16,24,32,16 --streams 2,3 --frames 960 > gpurun_out/batch_big.jsonl 2> gpurun_out/batch_big.err || { tail -5 gpurun_out/batch_big.err; exit 1; }
cat gpurun_out/batch_big.jsonl
