#!/bin/bash
# A/B: 48-output Winograd kernel with one position per wave (libdenoise_hip_p1.so) -- isolated
# shapes (x6_micro) and the step
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_run.sh ab:-,p1 > gpurun_out/p1ab.log 2>&1 || { tail -20 gpurun_out/p1ab.log; exit 1; }
grep -E '48->' gpurun_out/p1ab.log
LIBS="- p1" OPS="fwd3 dgrad3" bash tools/probes/r5_libab.sh
