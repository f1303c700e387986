#!/bin/bash
# deconv forward: per-fragment weight reads + three-deep input prefetch (default) vs dcold
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py \
  tests/test_gpu_parity.py -m gpu -k "deconv or unet or n2n" > gpurun_out/t_l.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/t_l.log | head -30; exit 1; }
tail -1 gpurun_out/t_l.log
for r in 1 2; do
  for v in "" _dcold; do
    DN_LIB_PATH=image_denoising_amd/libdenoise_hip$v.so OPS=deconv_x6 timeout -k 10 120 python -u tools/bench_ops.py 2>&1 | grep deconv | sed "s/^/r$r ${v:-new}: /" || exit 1
  done
done
B=image_denoising_amd/libdenoise_hip
bash tools/gpu_ab.sh "X=1 --" "DN_LIB_PATH=${B}_dcold.so --" "X=1 --" "DN_LIB_PATH=${B}_dcold.so --"
