#!/bin/bash
# adapter backward + wgrad DMA addressing A/B (libdenoise_hip_gen.so = per-stage addressing)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
GEN=image_denoising_amd/libdenoise_hip_gen.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_adapter.py \
  tests/test_gpu_bf16.py tests/test_gpu_x6.py -m gpu -k "adapter or finetune or weight" > gpurun_out/t_d.log 2>&1 \
  || { tail -30 gpurun_out/t_d.log; exit 1; }
tail -1 gpurun_out/t_d.log
timeout -k 10 200 python -u tools/x6_micro.py 2>&1 | grep wgrad
DN_LIB_PATH=$GEN timeout -k 10 200 python -u tools/x6_micro.py 2>&1 | grep wgrad | sed 's/^/gen: /'
bash tools/gpu_ab.sh "X=1 --" "DN_LIB_PATH=$GEN --" "X=1 --" "X=1 -- --mode finetune --precision bf16" || exit 1
PROF_STEPS=3 bash tools/profile.sh ft_bf16_r2d --mode finetune --precision bf16 2>&1 | grep -E "adapter|total" 
