#!/bin/bash
# mid-stage x-tile split (default) vs after the stage's MFMAs (nomidx): tests, micro, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_parity.py \
  -m gpu > gpurun_out/t_p.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/t_p.log | head -30; exit 1; }
tail -1 gpurun_out/t_p.log
for r in 1 2; do
  for v in "" _nomidx; do
    DN_LIB_PATH=image_denoising_amd/libdenoise_hip$v.so timeout -k 10 200 python -u tools/x6_micro.py 2>&1 | grep -E "fwd|dgrad" | sed "s/^/r$r ${v:-midx}: /" || exit 1
  done
done
B=image_denoising_amd/libdenoise_hip
bash tools/gpu_ab.sh "X=1 --" "DN_LIB_PATH=${B}_nomidx.so --" "X=1 --" "DN_LIB_PATH=${B}_nomidx.so --"
