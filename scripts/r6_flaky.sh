#!/bin/bash
# the whole GPU suite twice (flakiness check), then smoke
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  scripts/gpu_step.sh 600 fl_$i.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
  grep -q "passed" gpurun_out/fl_$i.log && ! grep -q "failed" gpurun_out/fl_$i.log || { echo "RUN $i FAILED"; tail -30 gpurun_out/fl_$i.log; exit 1; }
done
scripts/gpu_step.sh 300 fl_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
grep -h "passed\|smoke" gpurun_out/fl_1.log gpurun_out/fl_2.log gpurun_out/fl_smoke.log
