#!/bin/bash
# Build a variant of ONE kernel source against the base objects:
#   scripts/bv1.sh <name> <file.hip> <extra hipcc flags...>
# -> juicefs_amd/lib/libjfsgpu_<name>.so (select with JFS_GPU_LIB=...)
set -e
name=$1; shift; src=$1; shift
cd "$(dirname "$0")/../juicefs_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../build/v1_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable "$@" -c $src -o ../build/v1_$name/${src%.hip}.o
objs=""
for f in *.hip; do
  if [ "$f" = "$src" ]; then objs="$objs ../build/v1_$name/${f%.hip}.o"; else objs="$objs ../build/${f%.hip}.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../lib/libjfsgpu_$name.so $objs -lpthread
echo built ../lib/libjfsgpu_$name.so
