#!/bin/bash
# Round-end evidence on the GPU box: bench lines, rocprofv3 kernel-trace stats
# of the bench command, PMC traffic passes.  Everything lands in gpurun_out/prof/.
# usage: scripts/profile_round.sh [lz4|zstd|all]
set -e
what=${1:-all}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
if [ "$what" = lz4 ] || [ "$what" = all ]; then
  timeout -k 10 400 python bench.py > $O/bench_lz4.json 2> $O/bench_lz4.err
  tail -1 $O/bench_lz4.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_lz4 -o kt --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras --no-host-path > $O/kt_lz4.log 2>&1
  find $O/kt_lz4 -name '*kernel_stats.csv' -exec cp {} $O/lz4_kernel_stats.csv \;
  cat $O/lz4_kernel_stats.csv
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o pf --output-format csv -- python scripts/prof_run.py 4096 1 T > $O/pf.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o pw --output-format csv -- python scripts/prof_run.py 4096 1 T > $O/pw.log 2>&1
  python scripts/traffic.py $(find $O/pf -name '*counter_collection.csv' | head -1) $(find $O/pw -name '*counter_collection.csv' | head -1) lz4_decode_kernel 4096 4194304 $O/traffic.json
fi
if [ "$what" = zstd ] || [ "$what" = all ]; then
  timeout -k 10 300 python bench.py --codec zstd > $O/bench_zstd.json 2> $O/bench_zstd.err
  tail -1 $O/bench_zstd.json
  # (libzstd is not loaded under the profiler: the conda libzstd clashes with the
  # profiler's own; the frames come from a cache written by an unprofiled run)
  timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > $O/zcache.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_zstd -o kt --output-format csv -- python scripts/prof_run.py 4096 5 T zstd > $O/kt_zstd.log 2>&1
  find $O/kt_zstd -name '*kernel_stats.csv' -exec cp {} $O/zstd_kernel_stats.csv \;
  cat $O/zstd_kernel_stats.csv
fi
