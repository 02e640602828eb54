#!/bin/bash
# Build a library variant with one source file replaced:
#   scripts/bvfile.sh <name> <file.hip in csrc> <path/to/alternative source> [hipcc flags...]
#   -> juicefs_amd/lib/libjfsgpu_<name>.so
set -e
name=$1; tgt=$2; shift 2; srcf=$(readlink -f "$1"); shift
cd "$(dirname "$0")/../juicefs_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../build/vf_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -I. -I../../include "$@" -x hip -c "$srcf" -o ../build/vf_$name/${tgt%.hip}.o
objs=""
for f in *.hip; do
  if [ "$f" = "$tgt" ]; then objs="$objs ../build/vf_$name/${tgt%.hip}.o"; else objs="$objs ../build/${f%.hip}.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../lib/libjfsgpu_$name.so $objs -lpthread
echo built ../lib/libjfsgpu_$name.so
