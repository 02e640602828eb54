#!/bin/bash
# Build a variant from an alternative lz4_decode.hip source file:
#   scripts/bvsrc.sh <name> <path/to/lz4_decode.hip> [hipcc flags...]  -> juicefs_amd/lib/libjfsgpu_<name>.so
set -e
name=$1; shift; srcf=$(readlink -f "$1"); shift
cd "$(dirname "$0")/../juicefs_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../build/v1_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -I. -I../../include "$@" -x hip -c "$srcf" -o ../build/v1_$name/lz4_decode.o
objs=""
for f in *.hip; do
  if [ "$f" = lz4_decode.hip ]; then objs="$objs ../build/v1_$name/lz4_decode.o"; else objs="$objs ../build/${f%.hip}.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../lib/libjfsgpu_$name.so $objs -lpthread
echo built ../lib/libjfsgpu_$name.so
