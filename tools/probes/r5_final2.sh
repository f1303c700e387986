#!/bin/bash
# round 5 counters on the round's tree: FETCH / WRITE per launch of the bench step (-> the bench
# line's traffic) and one SQ pass per kernel
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_run.sh pmc:r5x_n2n sq:r5n:SQ_ACTIVE_INST_ANY+SQ_LDS_BANK_CONFLICT+SQ_LDS_IDX_ACTIVE+SQ_VALU_MFMA_BUSY_CYCLES+SQ_WAIT_ANY+SQ_WAIT_INST_ANY+SQ_INSTS_VALU+SQ_WAVE_CYCLES+GRBM_GUI_ACTIVE > gpurun_out/final2.log 2>&1 || { tail -20 gpurun_out/final2.log; exit 3; }
tail -40 gpurun_out/final2.log
