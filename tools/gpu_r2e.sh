#!/bin/bash
# carried x6 corrections: accuracy tests, micro A/B against libdenoise_hip_nocarry.so, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
NC=image_denoising_amd/libdenoise_hip_nocarry.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py \
  tests/test_gpu_parity.py -m gpu > gpurun_out/t_e.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/t_e.log | head -30; exit 1; }
tail -1 gpurun_out/t_e.log
timeout -k 10 200 python -u tools/x6_micro.py 2>&1 | grep -v wgrad
DN_LIB_PATH=$NC timeout -k 10 200 python -u tools/x6_micro.py 2>&1 | grep -v wgrad | sed 's/^/nocarry: /'
bash tools/gpu_ab.sh "X=1 --" "DN_LIB_PATH=$NC --" "X=1 --" "DN_LIB_PATH=$NC --"
PROF_STEPS=3 bash tools/profile.sh r2e_carry_sel2 2>&1 | head -14
