#!/bin/bash
# Build libjfsgpu_head.so: the committed (git HEAD) lz4_decode.hip against the current other objects,
# as the control in timing runs.
set -e
cd "$(dirname "$0")/../juicefs_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../build/v1_head
git show HEAD:juicefs_amd/csrc/lz4_decode.hip > ../build/v1_head/lz4_decode.hip
cp *.h *.cuh *.inc ../build/v1_head/ 2>/dev/null || true
cp ../../include/jfs_gpucodec.h ../build/v1_head/ 2>/dev/null || true
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -I. -I../../include "$@" -c ../build/v1_head/lz4_decode.hip -o ../build/v1_head/lz4_decode.o
objs=""
for f in *.hip; do
  if [ "$f" = lz4_decode.hip ]; then objs="$objs ../build/v1_head/lz4_decode.o"; else objs="$objs ../build/${f%.hip}.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../lib/libjfsgpu_head.so $objs -lpthread
echo built ../lib/libjfsgpu_head.so
