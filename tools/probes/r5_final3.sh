#!/bin/bash
# round 5 closing measurement set on the final tree: the default bench line (CPU baseline
# included), the secondary configurations, the one-rank RCCL torchrun line, rocprofv3 stats, the
# FETCH / WRITE per-launch summary (-> the bench line's traffic) and one SQ pass
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_run.sh bench configs torchrun1 stats:r5f pmc:r5y_n2n \
  sq:r5f:SQ_ACTIVE_INST_ANY+SQ_LDS_BANK_CONFLICT+SQ_LDS_IDX_ACTIVE+SQ_VALU_MFMA_BUSY_CYCLES+SQ_WAIT_ANY+SQ_WAIT_INST_ANY+SQ_INSTS_VALU+SQ_WAVE_CYCLES+GRBM_GUI_ACTIVE \
  > gpurun_out/final3.log 2>&1 || { tail -30 gpurun_out/final3.log; exit 3; }
tail -60 gpurun_out/final3.log
