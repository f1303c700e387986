#!/bin/bash
# round 5 closing check on the final tree: every GPU test, the smoke, the default bench line (CPU
# baseline and eval included) and rocprofv3 stats of the bench
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_run.sh tests smoke bench stats:r5z > gpurun_out/close.log 2>&1 || { tail -30 gpurun_out/close.log; exit 3; }
grep -E '^==|passed|failed|^\{' gpurun_out/close.log | cut -c1-300
