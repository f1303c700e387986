#!/bin/bash
# round 5: k_c3w6 / k_c3w6s with each fragment group's adds deferred past the next group's MFMAs
# -- x6 + pair-pass tests, isolated-shape A/B against the previous tree (libdenoise_hip_base.so),
# then a quick bench line for both libraries
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6.py tests/test_gpu_parity.py -m gpu -x -q -k "x6_forward or backward_data or pair_pixels or config1_full_size_step_vs or unit_gain" --timeout 300 --timeout-method thread > gpurun_out/w6def_tests.log 2>&1 || { grep -E "FAILED|assert|Error" gpurun_out/w6def_tests.log | head -20; exit 3; }
tail -1 gpurun_out/w6def_tests.log
for r in 1 2; do for v in base -; do
  lib=image_denoising_amd/libdenoise_hip.so; [ "$v" = "-" ] || lib=image_denoising_amd/libdenoise_hip_$v.so
  DN_LIB_PATH=$lib timeout -k 10 200 python -u - > gpurun_out/w6def_${v}_$r.log 2>&1 <<'PY' || { tail -5 gpurun_out/w6def_${v}_$r.log; exit 4; }
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
  sed "s/^/r$r $v: /" gpurun_out/w6def_${v}_$r.log | grep -v amdgpu.ids
done; done
for v in base -; do
  lib=image_denoising_amd/libdenoise_hip.so; [ "$v" = "-" ] || lib=image_denoising_amd/libdenoise_hip_$v.so
  DN_LIB_PATH=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/w6def_bench_$v.log 2>&1 || exit 5
  python3 - "$v" <<'PY'
import json, sys
for l in open(f"gpurun_out/w6def_bench_{sys.argv[1]}.log"):
    if l.startswith("{"): d = json.loads(l)
b = d["step_breakdown_ms"]; r = d["roofline"]
print(sys.argv[1], d["value"], d["ms_per_step"], "fwd3", b["fwd3"], "dgrad3", b["dgrad3"], "fwd3sel", b["fwd3sel"], "dominant", r["avg_launch_ms"], r["frac"], "weighted", r["weighted_frac"])
PY
done
