#!/bin/bash
# pinned in-group hi adds (default) vs sunk adds (nopin): x6 tests, interleaved micro, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py \
  -m gpu > gpurun_out/t_h.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/t_h.log | head -30; exit 1; }
tail -1 gpurun_out/t_h.log
for r in 1 2; do
  for v in "" _nopin; do
    L=image_denoising_amd/libdenoise_hip$v.so
    DN_LIB_PATH=$L timeout -k 10 200 python -u tools/x6_micro.py 2>&1 | grep -E "fwd|dgrad" | sed "s/^/r$r ${v:-pin}: /" || exit 1
  done
done
bash tools/gpu_ab.sh "X=1 --" "DN_LIB_PATH=image_denoising_amd/libdenoise_hip_nopin.so --" "X=1 --" "DN_LIB_PATH=image_denoising_amd/libdenoise_hip_nopin.so --"
