#!/bin/bash
# Build the working tree's librt_amd.so with extra compiler flags (e.g. -DRT_WV=1) into
# raytracer.js_amd/lib/librt_amd_NAME.so, for same-box A/B runs (tools/ab_libs.sh).
set -eu
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
mkdir -p "$TMP/include" "$TMP/pkg"
cp "$ROOT/include/rt.h" "$TMP/include/"
cp -r "$ROOT/raytracer.js_amd/csrc" "$TMP/pkg/"
cp "$ROOT/raytracer.js_amd/Makefile" "$TMP/pkg/"
make -s -j8 -C "$TMP/pkg" COMMON="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I../include -Icsrc -Wall -Wno-unused-function $*" >/dev/null
cp "$TMP/pkg/lib/librt_amd.so" "$ROOT/raytracer.js_amd/lib/librt_amd_$NAME.so"
rm -rf "$TMP"
echo "built $* -> raytracer.js_amd/lib/librt_amd_$NAME.so"
