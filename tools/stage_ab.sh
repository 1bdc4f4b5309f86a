#!/bin/bash
# Saturated (3-stream bench) cost of stages: libsift_hip variants with stages
# compiled out (-DSIFT_SKIP_STAGES=list; results wrong by construction) run
# under bench.py via SIFT_HIP_LIB.  "none" = the full pipeline.
#   tools/stage_ab.sh build      (here, hipcc)      tools/stage_ab.sh run   (GPU box)
set -e
cd "$(dirname "$0")/.."
OUT=another-cuda-sift_amd/lib/variants
KP="refine,orientation,select,bucket_count,bucket_scan,bucket_scatter,bucket_rank,descriptor"
declare -A V
V[no_desc]="descriptor"
V[no_ori]="orientation"
V[no_refine]="refine"
V[pyr_only]="extrema,$KP"
V[no_kp]="$KP"
V[blur_o0_only]="blur_o1,blur_o2,extrema,$KP"
V[init_only]="blur_o0,blur_o1,blur_o2,extrema,$KP"
if [ "$1" = build ]; then
  mkdir -p $OUT
  HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Ianother-cuda-sift_amd/csrc"
  OBJS=$(ls another-cuda-sift_amd/lib/obj/*.o | grep -v detector.o)
  for v in "${!V[@]}"; do
    /opt/rocm/bin/hipcc $HIPFLAGS "-DSIFT_SKIP_STAGES=\"${V[$v]}\"" -c another-cuda-sift_amd/csrc/detector.hip -o $OUT/detector_$v.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsift_hip_$v.so $OBJS $OUT/detector_$v.o -Wl,-soname,libsift_hip.so
  done
else
  export TMPDIR=/tmp
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/stage_ab_none.json 2>/dev/null
  for v in "${!V[@]}"; do
    SIFT_HIP_LIB=$PWD/$OUT/libsift_hip_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/stage_ab_$v.json 2>/dev/null || exit 1
  done
fi
