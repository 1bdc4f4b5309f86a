#!/bin/bash
# Build the working tree's libsift_hip.so with a source edit (a sed script over
# one csrc file: constants of a measured alternative) into ab/NAME.so -- A/B
# variants without compile-time knobs in the product sources.
# Usage: tools/ab_sed.sh NAME FILE 'SED-SCRIPT'
set -e
NAME=$1; FILE=$2; SCRIPT=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cp -r "$ROOT/Makefile" "$ROOT/include" "$TMP/"
mkdir -p "$TMP/another-cuda-sift_amd" && cp -r "$ROOT/another-cuda-sift_amd/csrc" "$TMP/another-cuda-sift_amd/"
sed -i "$SCRIPT" "$TMP/another-cuda-sift_amd/csrc/$FILE"
if cmp -s "$ROOT/another-cuda-sift_amd/csrc/$FILE" "$TMP/another-cuda-sift_amd/csrc/$FILE"; then echo "sed changed nothing"; exit 1; fi
make -C "$TMP" -j8 another-cuda-sift_amd/lib/libsift_hip.so EXTRA_HIPFLAGS="-DSIFT_AB_SED" > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
mkdir -p "$ROOT/ab"
cp "$TMP/another-cuda-sift_amd/lib/libsift_hip.so" "$ROOT/ab/$NAME.so"
rm -rf "$TMP"
echo "ab/$NAME.so <- working tree + sed '$SCRIPT' on $FILE"
