#!/bin/bash
# round 5 measurement set on the round's tree: the default bench line (CPU baseline included),
# secondary configurations, the one-rank RCCL torchrun line, then rocprofv3 stats
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_run.sh bench configs torchrun1 stats:r5 || exit $?
