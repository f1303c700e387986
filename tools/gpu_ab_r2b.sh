#!/bin/bash
# one-box A/B of the round-2 kernel variants: 16-row 48-channel tiles (DN_X6_H4), scalar vs
# packed fp32 adds (libdenoise_hip_pk.so), pipelined bf16 3x3 + x6 head in the bf16 base
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PK=image_denoising_amd/libdenoise_hip_pk.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py \
  tests/test_gpu_bf16.py tests/test_gpu_adapter.py -m gpu > gpurun_out/tx6.log 2>&1 || { tail -30 gpurun_out/tx6.log; exit 1; }
tail -1 gpurun_out/tx6.log
timeout -k 10 200 python -u tools/x6_micro.py > gpurun_out/m_def.log 2>&1 || exit 1
DN_X6_H4=0 timeout -k 10 200 python -u tools/x6_micro.py > gpurun_out/m_h40.log 2>&1 || exit 1
DN_LIB_PATH=$PK timeout -k 10 200 python -u tools/x6_micro.py > gpurun_out/m_pk.log 2>&1 || exit 1
paste gpurun_out/m_def.log gpurun_out/m_h40.log gpurun_out/m_pk.log | awk -F'\t' '{print $1; print "   h4=0: " $2; print "   pk:   " $3}'
bash tools/gpu_ab.sh "DN_X6_H4=1 --" "DN_X6_H4=0 --" "DN_LIB_PATH=$PK --" "DN_X6_H4=1 --" \
  "DN_BF16_PIPE=1 -- --mode finetune --precision bf16" \
  "DN_BF16_PIPE=0 DN_BF16_HEAD_X6=0 DN_BF16_DECONV_X6=0 -- --mode finetune --precision bf16" \
  "DN_BF16_PIPE=1 DN_BF16_HEAD_X6=0 -- --mode finetune --precision bf16" || exit 1
bash tools/pmc_sq.sh wgrad > gpurun_out/pmcw1.txt 2>&1 || exit 1
CTRS="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES" \
  bash tools/pmc_sq.sh wgrad wgrad2 > gpurun_out/pmcw2.txt 2>&1
cat gpurun_out/pmcw1.txt gpurun_out/pmcw2.txt
