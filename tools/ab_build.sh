#!/bin/bash
# Build libsift_hip.so of git revision REV into ab/NAME.so (for A/B runs on the
# GPU box: SIFT_HIP_LIB=ab/NAME.so python tools/batch_sweep.py ...).
# Usage: tools/ab_build.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" Makefile include another-cuda-sift_amd/csrc | tar -x -C "$TMP"
make -C "$TMP" -j8 another-cuda-sift_amd/lib/libsift_hip.so > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
mkdir -p "$ROOT/ab"
cp "$TMP/another-cuda-sift_amd/lib/libsift_hip.so" "$ROOT/ab/$NAME.so"
rm -rf "$TMP"
echo "ab/$NAME.so <- $REV"
