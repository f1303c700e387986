#!/bin/bash
# interleaved micro A/B of the B-fragment look-ahead (default 2, look1, look3)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
  for v in "" _look1 _look3; do
    L=image_denoising_amd/libdenoise_hip$v.so
    DN_LIB_PATH=$L timeout -k 10 200 python -u tools/x6_micro.py 2>&1 | grep -E "fwd|dgrad" | sed "s/^/r$r ${v:-look2}: /" || exit 1
  done
done
