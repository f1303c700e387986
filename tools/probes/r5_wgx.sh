#!/bin/bash
# round 5: XCD-aligned wgrad split counts -- weight tests, isolated wgrad shapes A/B against
# libdenoise_hip_base.so, bench lines for both
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6.py tests/test_gpu_parity.py -m gpu -x -q -k "weight or unit_gain or config1_full_size_step_vs" --timeout 300 --timeout-method thread > gpurun_out/wgx_tests.log 2>&1 || { grep -E "FAILED|assert|Error" gpurun_out/wgx_tests.log | head -20; exit 3; }
tail -1 gpurun_out/wgx_tests.log
for r in 1 2; do for v in base -; do
  lib=image_denoising_amd/libdenoise_hip.so; [ "$v" = "-" ] || lib=image_denoising_amd/libdenoise_hip_$v.so
  DN_LIB_PATH=$lib timeout -k 10 200 python -u - > gpurun_out/wgx_${v}_$r.log 2>&1 <<'PY' || { tail -5 gpurun_out/wgx_${v}_$r.log; exit 4; }
import os, sys
sys.path.insert(0, os.getcwd())
from tools.x6_shapes import wgrad
out = []
for cin, cout, H in ((96, 96, 128), (144, 96, 64), (96, 96, 64), (144, 96, 32), (96, 96, 32)):
    ms = wgrad(cin, cout, H, True)
    fl = 2.0 * 64 * H * H * cin * cout * 9
    out.append(f"{cin}->{cout}@{H} {ms:.3f}ms/{fl / ms / 1e9 / (2500 / 6):.3f}")
print(" ".join(out))
PY
  sed "s/^/r$r $v: /" gpurun_out/wgx_${v}_$r.log | grep -v amdgpu.ids
done; done
for v in base -; do
  lib=image_denoising_amd/libdenoise_hip.so; [ "$v" = "-" ] || lib=image_denoising_amd/libdenoise_hip_$v.so
  DN_LIB_PATH=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/wgx_bench_$v.log 2>&1 || exit 5
  python3 - "$v" <<'PY'
import json, sys
for l in open(f"gpurun_out/wgx_bench_{sys.argv[1]}.log"):
    if l.startswith("{"): d = json.loads(l)
b = d["step_breakdown_ms"]; r = d["roofline"]
print(sys.argv[1], d["value"], d["ms_per_step"], "fwd3", b["fwd3"], "dgrad3", b["dgrad3"], "wgrad3", b["wgrad3"], "reduce", b["reduce"], "weighted", r["weighted_frac"])
PY
done
