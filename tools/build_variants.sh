#!/bin/bash
# Build libttship variants that differ only in decoder_persist.hip compile flags:
#   tools/build_variants.sh name1 "-DX=1" name2 "-DX=2" ...   ->  tools/var/lib_<name>.so
# Select one at run time with TTSHIP_LIB=tools/var/lib_<name>.so (bench / tests).
set -e
cd "$(dirname "$0")/../tts_amd/csrc"
make -s ARCH=gfx950
mkdir -p ../../tools/var build/var
OTHERS=$(ls build/*.o | grep -v decoder_persist)
NAMES=""
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  NAMES="$NAMES $name"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../../include $flags \
    -c decoder_persist.hip -o build/var/dp_$name.o &
done
wait
for name in $NAMES; do
  o=build/var/dp_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/var/lib_$name.so $OTHERS $o
done
ls -la ../../tools/var
