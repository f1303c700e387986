#!/bin/bash
# x6 nin head: UNet parity (both precisions), smoke, bench A/B (DN_X6_HEAD)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "unet or n2n or config1" -x -q --timeout 200 --timeout-method thread > gpurun_out/head6_t.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/head6_t.log; grep -E "^E " gpurun_out/head6_t.log | head
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh "DN_X6_DECONV=0 -- --steps 20 --warmup 3" "DN_X6_DECONV=1 -- --steps 20 --warmup 3"
