#!/bin/bash
# the driver's round-end GPU steps: the GPU suite and smoke(), twice
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for k in 1 2; do
  scripts/gpu_step.sh 600 fc_t$k.log python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread || exit 1
  scripts/gpu_step.sh 300 fc_s$k.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
done
tail -n 1 gpurun_out/fc_t1.log gpurun_out/fc_t2.log gpurun_out/fc_s1.log gpurun_out/fc_s2.log
