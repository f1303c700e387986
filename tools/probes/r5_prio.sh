#!/bin/bash
# stream-priority A/B of the step: the no-grad pass's stream at high priority (trainer), the
# backward's weight-gradient stream at high priority (libdenoise_hip_prhi.so)
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
: > gpurun_out/prio.log
for r in 1 2 3; do
  for v in base sidehi prhi; do
    lib=image_denoising_amd/libdenoise_hip.so; sp=0
    [ $v = prhi ] && lib=image_denoising_amd/libdenoise_hip_prhi.so
    [ $v = sidehi ] && sp=-1
    DN_LIB_PATH=$lib DN_STEP_SIDE_PRIO=$sp timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eval > gpurun_out/prio_${v}_$r.log 2>&1 || exit $?
    echo "r$r $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prio_${v}_$r.log | head -1)" >> gpurun_out/prio.log
  done
done
cat gpurun_out/prio.log
