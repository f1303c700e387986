#!/bin/bash
# k_wgrad3p ablations (timing-only builds, DN_WG_ABL_*): what bounds the weight-gradient stage loop
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_run.sh ab:-,wnos,wnold,wnobar > gpurun_out/wgabl.log 2>&1 || { tail -20 gpurun_out/wgabl.log; exit 1; }
grep -E 'wgrad' gpurun_out/wgabl.log
