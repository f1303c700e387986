#!/bin/bash
# up1 concat stride: 128 in forward-only plans, 100 with a backward (default) vs all-100 / all-128
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bf16.py \
  -m gpu > gpurun_out/t_n.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/t_n.log | head -30; exit 1; }
tail -1 gpurun_out/t_n.log
bash tools/gpu_ab.sh "X=1 --" "DN_C1S_ALIGN=4 --" "DN_C1S_ALIGN=32 --" "X=1 --" "DN_C1S_ALIGN=4 --" "DN_C1S_ALIGN=32 --" \
  "X=1 -- --mode finetune --precision bf16" "DN_C1S_ALIGN=4 -- --mode finetune --precision bf16"
