#!/bin/bash
# round 5: where k_c3w6's time goes -- ablation builds (timing only, wrong results): abl_t = V
# built for the first chunk only, abl_w = no weight loads in the stage loop, abl_tw = both
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2; do for v in - abl_t abl_w abl_tw; do
  lib=image_denoising_amd/libdenoise_hip.so; [ "$v" = "-" ] || lib=image_denoising_amd/libdenoise_hip_$v.so
  DN_LIB_PATH=$lib timeout -k 10 200 python -u - > gpurun_out/w6abl_${v}_$r.log 2>&1 <<'PY' || { tail -5 gpurun_out/w6abl_${v}_$r.log; exit 4; }
import os, sys
sys.path.insert(0, os.getcwd())
from tools.x6_shapes import fwd, dgrad
out = []
for op, cin, cout, H in (("fwd", 96, 96, 256), ("fwd", 96, 96, 128), ("fwd", 100, 96, 256), ("dgrad", 96, 96, 128), ("fwd", 144, 96, 128)):
    ms = (fwd if op == "fwd" else dgrad)(cin, cout, H, True)
    fl = 2.0 * 64 * H * H * cin * cout * 9
    out.append(f"{op}{cin}->{cout}@{H} {ms:.3f}ms/{fl / ms / 1e9 / (2500 / 6):.3f}")
print(" ".join(out))
PY
  sed "s/^/r$r $v: /" gpurun_out/w6abl_${v}_$r.log | grep -v amdgpu.ids
done; done
