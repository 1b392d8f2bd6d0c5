#!/bin/bash
# Build librt_amd.so from a git revision (default HEAD) into raytracer.js_amd/lib/librt_amd_ref.so,
# the "ref" arm of tools/ab_sweep.sh (same-box A/B against the working tree's build).
set -eu
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
mkdir -p "$TMP/include" "$TMP/pkg/csrc"
git -C "$ROOT" show "$REV:include/rt.h" > "$TMP/include/rt.h"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" raytracer.js_amd/csrc/); do
  git -C "$ROOT" show "$REV:$f" > "$TMP/pkg/csrc/$(basename "$f")"
done
git -C "$ROOT" show "$REV:raytracer.js_amd/Makefile" > "$TMP/pkg/Makefile"
make -s -j8 -C "$TMP/pkg" >/dev/null
cp "$TMP/pkg/lib/librt_amd.so" "$ROOT/raytracer.js_amd/lib/librt_amd_ref.so"
rm -rf "$TMP"
echo "built $REV -> raytracer.js_amd/lib/librt_amd_ref.so"
