#!/bin/bash
# Marginal cost of each stage under the saturated multi-stream bench: build
# libsift_hip variants with stages compiled out (-DSIFT_SKIP_STAGES, results
# wrong by construction) and run bench.py against each (SIFT_HIP_LIB).
#   tools/stage_ab.sh build      (here, hipcc)      tools/stage_ab.sh run   (GPU box)
set -e
cd "$(dirname "$0")/.."
OUT=another-cuda-sift_amd/lib/variants
VARIANTS="descriptor orientation extrema refine blur_o1,blur_o2 blur_o0"
if [ "$1" = build ]; then
  mkdir -p $OUT
  HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Ianother-cuda-sift_amd/csrc"
  OBJS=$(ls another-cuda-sift_amd/lib/obj/*.o | grep -v detector.o)
  for v in $VARIANTS; do
    /opt/rocm/bin/hipcc $HIPFLAGS "-DSIFT_SKIP_STAGES=\"$v\"" -c another-cuda-sift_amd/csrc/detector.hip -o $OUT/detector_$v.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsift_hip_$v.so $OBJS $OUT/detector_$v.o -Wl,-soname,libsift_hip.so
  done
else
  export TMPDIR=/tmp
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/stage_ab_none.json 2>/dev/null
  for v in $VARIANTS; do
    SIFT_HIP_LIB=$PWD/$OUT/libsift_hip_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/stage_ab_$v.json 2>/dev/null || exit 1
  done
fi
