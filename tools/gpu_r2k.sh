#!/bin/bash
# bf16 base (configs[4]) weight DMA as buffer loads (default) vs global_load_lds (bfold); bf16
# tests; SQ counters of the dominant x6 kernel
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py \
  -m gpu > gpurun_out/t_k.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/t_k.log | head -30; exit 1; }
tail -1 gpurun_out/t_k.log
O=image_denoising_amd/libdenoise_hip_bfold.so
bash tools/gpu_ab.sh "X=1 -- --mode finetune --precision bf16" "DN_LIB_PATH=$O -- --mode finetune --precision bf16" \
  "X=1 -- --mode finetune --precision bf16" "DN_LIB_PATH=$O -- --mode finetune --precision bf16" || exit 1
bash tools/pmc_sq.sh x6 x6_r2k
