#!/bin/bash
# Build the working tree's libsift_hip.so with extra compiler flags (tuning
# knobs, e.g. -DSIFT_BLUR_TH=32 or -DSIFT_DESC_PRECISE=1) into ab/NAME.so.
# Usage: tools/ab_variant.sh NAME "FLAGS"
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cp -r "$ROOT/Makefile" "$ROOT/include" "$TMP/"
mkdir -p "$TMP/another-cuda-sift_amd" && cp -r "$ROOT/another-cuda-sift_amd/csrc" "$TMP/another-cuda-sift_amd/"
make -C "$TMP" -j8 another-cuda-sift_amd/lib/libsift_hip.so EXTRA_HIPFLAGS="$FLAGS" > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
mkdir -p "$ROOT/ab"
cp "$TMP/another-cuda-sift_amd/lib/libsift_hip.so" "$ROOT/ab/$NAME.so"
rm -rf "$TMP"
echo "ab/$NAME.so <- working tree $FLAGS"
