#!/bin/bash
# up1 concat stride 128 (default) vs 100 (DN_C1S_ALIGN=4): GPU suite, bench A/B, kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_m.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/t_m.log | head -30; exit 1; }
tail -1 gpurun_out/t_m.log
bash tools/gpu_ab.sh "X=1 --" "DN_C1S_ALIGN=4 --" "X=1 --" "DN_C1S_ALIGN=4 --" "X=1 -- --mode finetune --precision bf16" "DN_C1S_ALIGN=4 -- --mode finetune --precision bf16" || exit 1
DN_STEP_STREAMS=0 DN_BWD_STREAMS=0 PROF_STEPS=3 bash tools/profile.sh c1s128_1stream 2>&1 | head -16
