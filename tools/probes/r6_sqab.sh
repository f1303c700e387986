#!/bin/bash
# SQ LDS-conflict counters of two libraries (default, prev) on the bench step, one pass each
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C=${CTRS:-SQ_LDS_BANK_CONFLICT+SQ_LDS_IDX_ACTIVE+SQ_WAVE_CYCLES+SQ_WAIT_ANY+SQ_WAIT_INST_ANY+SQ_VALU_MFMA_BUSY_CYCLES+GRBM_GUI_ACTIVE}
bash tools/gpu_run.sh sq:r6new:$C > gpurun_out/sq_r6new.txt 2>&1 || exit $?
DN_LIB_PATH=image_denoising_amd/libdenoise_hip_prev.so bash tools/gpu_run.sh sq:r6prev:$C > gpurun_out/sq_r6prev.txt 2>&1 || exit $?
grep -E "k_c3w6<|k_c3w6s" gpurun_out/sq_r6new.txt | sed 's/^/new  /'
grep -E "k_c3w6<|k_c3w6s" gpurun_out/sq_r6prev.txt | sed 's/^/prev /'
