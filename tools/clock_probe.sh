#!/bin/bash
# Sample the GPU clocks while the dominant 3x3 conv kernel runs back to back for ~15 s.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 120 python - > gpurun_out/clk_load.log 2>&1 <<'PY' &
import sys, time, torch
sys.path.insert(0, ".")
from bench import time_dominant_kernel
t0 = time.time()
while time.time() - t0 < 15:
    ms, fl = time_dominant_kernel(64, 256, 256, torch.device("cuda"), reps=20)
    print(f"{ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s", flush=True)
PY
BP=$!
sleep 4
for i in $(seq 1 12); do
  (timeout 10 rocm-smi --showclocks 2>/dev/null | grep -E "sclk" | head -2) >> gpurun_out/clocks.log
  (timeout 10 rocm-smi --showpower 2>/dev/null | grep -iE "Current Socket" | head -1) >> gpurun_out/clocks.log
  sleep 0.5
done
wait $BP; rc=$?
sort gpurun_out/clocks.log | uniq -c | sort -rn | head -20
tail -3 gpurun_out/clk_load.log
exit $rc
