#!/bin/bash
# x6 weight-gradient check: kernel tests, UNet gradient parity, bench A/B (DN_X6_WGRAD)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py -k backward_weight -x -v --timeout 120 --timeout-method thread > gpurun_out/wgx6_t1.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/wgx6_t1.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "x6" -x -q --timeout 200 --timeout-method thread > gpurun_out/wgx6_t2.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/wgx6_t2.log; grep -E "^E " gpurun_out/wgx6_t2.log | head
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh "DN_X6_WGRAD=0 -- --steps 20 --warmup 3" "DN_X6_WGRAD=1 -- --steps 20 --warmup 3"
