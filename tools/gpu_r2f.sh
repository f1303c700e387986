#!/bin/bash
# interleaved micro A/B: carry (default) / nocarry / carry with per-block k_c3x6h (hpb)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" _nocarry _hpb; do
    L=image_denoising_amd/libdenoise_hip$v.so
    DN_LIB_PATH=$L timeout -k 10 200 python -u tools/x6_micro.py 2>&1 | grep -E "fwd|dgrad" | sed "s/^/r$r ${v:-carry}: /" || exit 1
  done
done
