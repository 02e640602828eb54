#!/bin/bash
# host_path LZ4 decode/encode rate of library variants (2 runs each): scripts/hostpath_variants.sh name...
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  for r in 1 2; do
    JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/hostpath.py 4096 > gpurun_out/hp_$v.json || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['lz4_decompress']['value'],2), round(d['lz4_compress']['value'],2), flush=True)" gpurun_out/hp_$v.json $v
  done
done
