#!/bin/bash
# host_path LZ4 decode of library variants, interleaved reps: scripts/hostpath_reps.sh REPS name...
cd "$GRAFT_REPO_ROOT"
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
    JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/hostpath.py 4096 > gpurun_out/hp_$v.json || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['lz4_decompress']['value'],2), flush=True)" gpurun_out/hp_$v.json $v
  done
done
