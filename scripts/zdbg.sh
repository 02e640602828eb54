#!/bin/bash
# per-kernel times of the Zstd decode (rocprofv3 kernel trace), N frames
set -e
N=${1:-512}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python scripts/prof_run.py $N 0 T zstd
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/zdbg -o run -- python3 scripts/prof_run.py $N 2 T zstd
