#!/bin/bash
# Build an A/B variant of the library: recompile the named sources with extra
# compile-time flags and link them with the default objects (build/*.o).
#   tools/build_variant.sh NAME "FLAGS" src1.hip [src2.hip ...]  -> ab/NAME.so
set -eu
cd "$(dirname "$0")/../algo-dsp_amd"
name=$1; flags=$2; shift 2
make -s >/dev/null
mkdir -p ../${ABDIR:-ab}/$name
objs=""
for src in "$@"; do
  b=$(basename "$src"); b=${b%.*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-parameter $flags -c csrc/$src -o ../${ABDIR:-ab}/$name/$b.o
  objs="$objs $b.o"
done
link=""
for o in build/*.o; do
  skip=0; for x in $objs; do [ "$(basename $o)" = "$x" ] && skip=1; done
  [ $skip = 0 ] && link="$link $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined $link ../${ABDIR:-ab}/$name/*.o -ldl -lpthread -o ../${ABDIR:-ab}/$name.so
echo built ${ABDIR:-ab}/$name.so
