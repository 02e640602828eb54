#!/bin/bash
# FETCH_SIZE and L2 hit/miss of the LZ4 decode kernel per library variant (two PMC passes each)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  for pass in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    tag=$(echo $pass | cut -c1-8)
    JFS_GPU_LIB=$lib JFS_NOVERIFY=1 timeout -s KILL 90 rocprofv3 --pmc $pass -d gpurun_out/tcc_${v}_$tag -o p --output-format csv -- python scripts/prof_run.py 4096 1 T > gpurun_out/tcc_${v}_$tag.log 2>&1 || exit 1
    f=$(find gpurun_out/tcc_${v}_$tag -name '*counter_collection.csv' | head -1)
    echo "== $v $pass"; grep lz4_decode_kernel "$f" | awk -F, '{print $(NF-3), $(NF-2)}'
  done
done
