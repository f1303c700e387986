#!/bin/bash
# round 5: k_wgrad3p B look-ahead (DN_WGP_BLA) and the 4-wave 48-output k_wgrad3q -- tests and
# same-box A/B against the round-4 library, the no-look-ahead build and DN_WGP_Q=0
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6.py -m gpu -x -q -k "weight" --timeout 240 --timeout-method thread > gpurun_out/wg_tests.log 2>&1 || { grep -E "FAILED|assert|Error" gpurun_out/wg_tests.log | head -20; exit 3; }
tail -1 gpurun_out/wg_tests.log
for r in 1 2; do for v in r4 nobla - q0; do
  lib=image_denoising_amd/libdenoise_hip.so; envq=1
  [ "$v" = "r4" ] || [ "$v" = "nobla" ] && lib=image_denoising_amd/libdenoise_hip_$v.so
  [ "$v" = "q0" ] && envq=0
  DN_WGP_Q=$envq DN_LIB_PATH=$lib timeout -k 10 200 python -u - > gpurun_out/wg_${v}_$r.log 2>&1 <<'PY' || { tail -5 gpurun_out/wg_${v}_$r.log; exit 4; }
import os, sys
sys.path.insert(0, os.getcwd())
from tools.x6_shapes import wgrad
out = []
for cin, cout, H in ((48, 48, 128), (48, 48, 64), (48, 48, 32), (96, 96, 128), (144, 96, 64), (96, 96, 64)):
    ms = wgrad(cin, cout, H, True)
    fl = 2.0 * 64 * H * H * cin * cout * 9
    out.append(f"{cin}->{cout}@{H} {ms:.3f}ms/{fl / ms / 1e9 / (2500 / 6):.3f}")
print(" ".join(out))
PY
  sed "s/^/r$r $v: /" gpurun_out/wg_${v}_$r.log | grep -v amdgpu.ids
done; done
bash tools/gpu_run.sh quick || exit 6
