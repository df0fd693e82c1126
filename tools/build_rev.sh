#!/bin/bash
# Build libttship.so from a git revision's sources (whole library, no mixing with this tree's
# objects) into tools/ab/lib_<name>.so, for same-box A/Bs (tools/gpu_ab.sh <rounds> <name>).
#   tools/build_rev.sh <rev> <name>
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2
tmp=$(mktemp -d)
git archive "$rev" tts_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/tts_amd/csrc" -j8 ARCH=gfx950
mkdir -p tools/ab
cp "$tmp/tts_amd/libttship.so" "tools/ab/lib_$name.so"
rm -rf "$tmp"
ls -la "tools/ab/lib_$name.so"
