#!/bin/bash
# bench lines of the secondary configurations (BASELINE configs[3], [4], the Structure_loss step,
# ImprovedUNet) at the current defaults -> gpurun_out/cfg_<name>.log
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 "$@" > gpurun_out/cfg_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/cfg_$name.log | cut -c1-200
  [ $rc -ne 0 ] && { tail -5 gpurun_out/cfg_$name.log; exit $rc; }
  return 0
}
run rgb --channels 3 --bs 32
run structure --mode structure
run finetune --mode finetune
run finetune_bf16 --mode finetune --precision bf16
run iunet --arch UNetImproved
