#!/bin/bash
# round 5: dec_conv1a's image channel(s) on the VALU in k_c3w6's epilogue (no tail chunk) --
# UNet-level parity tests, then both bench lines (previous tree = libdenoise_hip_base.so)
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_eval.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/thin_tests.log 2>&1 || { grep -E "FAILED|assert|Error" gpurun_out/thin_tests.log | head -20; exit 3; }
tail -1 gpurun_out/thin_tests.log
for r in 1 2; do for v in base -; do
  lib=image_denoising_amd/libdenoise_hip.so; [ "$v" = "-" ] || lib=image_denoising_amd/libdenoise_hip_$v.so
  DN_LIB_PATH=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/thin_bench_${v}_$r.log 2>&1 || exit 5
  python3 - "$v" "$r" <<'PY'
import json, sys
for l in open(f"gpurun_out/thin_bench_{sys.argv[1]}_{sys.argv[2]}.log"):
    if l.startswith("{"): d = json.loads(l)
b = d["step_breakdown_ms"]; r = d["roofline"]
sh = {s["shape"]: (s["kernel"], s["avg_launch_ms"], s["frac"]) for s in r["per_shape"] if s["shape"].startswith("97->96")}
print(sys.argv[2], sys.argv[1], d["value"], d["ms_per_step"], "fwd3", b["fwd3"], "dominant", r["kernel"][:40], r["avg_launch_ms"], r["frac"], "weighted", r["weighted_frac"], sh)
PY
done; done
