#!/bin/bash
# Round-5 session: the final profile set (tools/gpu_final.sh r5b bench), then
# the lane configuration A/B -- tools/dev_pipeline_time.py on ab/tp*.so, built
# by tools/ab_variant.sh with -DSIFT_AB_TPUT=1024|2048 [-DSIFT_AB_TPUT_EX=1]
# (single frames on a lane with the batch descriptor grid / extrema strips;
# the macros were removed after the A/B, profiles/round5/lane_tput_config_ab.jsonl).
set -o pipefail
bash tools/gpu_final.sh r5b bench || exit 1
for v in tp0 tp1k tp2k tp1kex tp0; do
  SIFT_HIP_LIB=ab/$v.so timeout -k 10 180 python tools/dev_pipeline_time.py >> gpurun_out/tput_ab.jsonl 2> gpurun_out/tput_ab.err || { echo "ab $v failed"; tail -5 gpurun_out/tput_ab.err; exit 1; }
done
cat gpurun_out/tput_ab.jsonl
