#!/bin/bash
# Micro-batch feasibility: C2 throughput of B-frame launch groups on S streams
# (tools/batch_sweep.py), small B.
set -o pipefail
timeout -k 10 400 python tools/batch_sweep.py --batches 1,2,3,4,6 --streams 2,3,4 --frames 300 > gpurun_out/mb_sweep.jsonl 2> gpurun_out/mb_sweep.err || { tail -5 gpurun_out/mb_sweep.err; exit 1; }
cat gpurun_out/mb_sweep.jsonl
