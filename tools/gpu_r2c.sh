#!/bin/bash
# bf16-base checks + profiles: tests, configs[4] bench and kernel stats, the N2N step's kernel
# stats with one stream (per-kernel durations not shared with a concurrent stream), and the
# dominant kernel alone under rocprofv3 (its average duration = the bench's roofline timing)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py \
  tests/test_gpu_adapter.py -m gpu > gpurun_out/t_bf16.log 2>&1 || { tail -30 gpurun_out/t_bf16.log; exit 1; }
tail -1 gpurun_out/t_bf16.log
bash tools/gpu_ab.sh "DN_BF16_HEAD_X6=1 -- --mode finetune --precision bf16" || exit 1
PROF_STEPS=3 bash tools/profile.sh ft_bf16_r2c --mode finetune --precision bf16 || exit 1
DN_STEP_STREAMS=0 DN_BWD_STREAMS=0 PROF_STEPS=3 bash tools/profile.sh n2n_1stream_r2c || exit 1
KERNEL=x6 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/dom_x6 -o run \
  -- python3 tools/dominant_kernel.py > gpurun_out/prof/dom_x6.log 2>&1 || exit 1
cat gpurun_out/prof/dom_x6/run_kernel_stats.csv | cut -c1-160
