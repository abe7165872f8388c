#!/bin/bash
# Build libnerf_amd.so from a git revision's sources into ab/<name>.so (A/B runs: NERF_AMD_LIB=ab/<name>.so).
# Usage: tools/build_rev.sh REV NAME
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
T=$(mktemp -d /tmp/rev_XXXX)
git archive "$REV" nerf-sys_amd include | tar -x -C "$T"
make -C "$T/nerf-sys_amd" -j8 > "$T/make.log" 2>&1 || { tail -20 "$T/make.log"; exit 1; }
mkdir -p ab && cp "$T/nerf-sys_amd/lib/libnerf_amd.so" "ab/$NAME.so"
rm -rf "$T"
echo "ab/$NAME.so from $REV"
