cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in base "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_zstd_gpu.py tests/test_zstd_split_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/zvt_$v.log 2>&1 || { echo "TESTS FAILED $v"; tail -20 gpurun_out/zvt_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/zvt_$v.log)"
done
bash scripts/time_zvariants.sh base "$@" base "$@"
