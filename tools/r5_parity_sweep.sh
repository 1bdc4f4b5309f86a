#!/bin/bash
# 200 fresh frames (100 per configuration) in both descriptor modes on the round-5 HEAD.
set -o pipefail
timeout -k 10 600 python3 -u tools/parity_sweep.py 100 > gpurun_out/parity_sweep_r5.json 2> gpurun_out/parity_sweep_r5.err || { tail -5 gpurun_out/parity_sweep_r5.err; exit 1; }
timeout -k 10 600 python3 -u tools/parity_sweep.py 100 --exact > gpurun_out/parity_sweep_exact_r5.json 2> gpurun_out/parity_sweep_exact_r5.err || { tail -5 gpurun_out/parity_sweep_exact_r5.err; exit 1; }
tail -c 600 gpurun_out/parity_sweep_r5.json; echo; tail -c 600 gpurun_out/parity_sweep_exact_r5.json
