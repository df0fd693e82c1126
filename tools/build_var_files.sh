#!/bin/bash
# Build one libttship variant whose listed sources are compiled with extra flags:
#   tools/build_var_files.sh <name> "<flags>" file1.hip [file2.hip ...]  ->  tools/var/lib_<name>.so
set -e
cd "$(dirname "$0")/../tts_amd/csrc"
make -s ARCH=gfx950
mkdir -p ../../tools/var build/var
name=$1; flags=$2; shift 2
objs=$(ls build/*.o)
for f in "$@"; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../../include $flags \
    -c $b.hip -o build/var/${name}_$b.o &
  objs=$(echo "$objs" | grep -v "build/$b.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/var/lib_$name.so $objs $(for f in "$@"; do echo build/var/${name}_$(basename $f .hip).o; done)
ls -la ../../tools/var/lib_$name.so
