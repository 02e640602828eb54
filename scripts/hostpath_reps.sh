#!/bin/bash
# host_path LZ4 decode of library variants, interleaved reps:
#   scripts/hostpath_reps.sh REPS NBLK name...   ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"
R=$1; N=$2; shift 2
for r in $(seq $R); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
    JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/hostpath.py $N > gpurun_out/hp_$v.json || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['lz4_decompress']['value'],2), flush=True)" gpurun_out/hp_$v.json $v $N
  done
done
