#!/bin/bash
# c2..c5 concat stride 160 in forward-only plans (default) vs the previous commit (prev)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_o.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/t_o.log | head -30; exit 1; }
tail -1 gpurun_out/t_o.log
P=image_denoising_amd/libdenoise_hip_prev.so
bash tools/gpu_ab.sh "X=1 --" "DN_LIB_PATH=$P --" "X=1 --" "DN_LIB_PATH=$P --" \
  "X=1 -- --mode finetune --precision bf16" "DN_LIB_PATH=$P -- --mode finetune --precision bf16" \
  "X=1 -- --mode finetune --precision bf16" "DN_LIB_PATH=$P -- --mode finetune --precision bf16"
