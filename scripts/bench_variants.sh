#!/bin/bash
# Time experimental library variants with the headline bench (no CPU legs).
# usage: scripts/bench_variants.sh name1 name2 ...   ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  r=$(JFS_GPU_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["roofline"]["kernel_ms"],2))')
  echo "$v $r"
done
