#!/bin/bash
# Build an experimental libjfsgpu variant: scripts/build_variant.sh <name> <extra hipcc flags...>
# -> juicefs_amd/lib/libjfsgpu_<name>.so (select with JFS_GPU_LIB=...)
set -e
name=$1; shift
cd "$(dirname "$0")/../juicefs_amd/csrc"
mkdir -p ../build/v_$name
objs=""
for f in *.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable "$@" -c $f -o ../build/v_$name/${f%.hip}.o &
  objs="$objs ../build/v_$name/${f%.hip}.o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../lib/libjfsgpu_$name.so $objs -lpthread
echo built ../lib/libjfsgpu_$name.so
