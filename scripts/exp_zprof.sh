cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 || exit 1
timeout -k 10 300 python scripts/zprof.py 4096 > gpurun_out/zp.log 2>&1; cat gpurun_out/zp.log | grep -v amdgpu
