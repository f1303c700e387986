#!/bin/bash
# ImprovedUNet step A/B of variant libraries (LIBS tags, '-' = default), OPS from the breakdown
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
LIBS=${LIBS:-"- base"}; OPS=${OPS:-"gn gnbwd"}
: > gpurun_out/iuab.log
for r in 1 2; do
  for v in $LIBS; do
    if [ "$v" = "-" ]; then lib=image_denoising_amd/libdenoise_hip.so; else lib=image_denoising_amd/libdenoise_hip_$v.so; fi
    DN_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --arch UNetImproved --steps 10 --warmup 2 --no-cpu-baseline --no-eval > gpurun_out/iuab_${v}_$r.log 2>&1 || exit $?
    python3 - gpurun_out/iuab_${v}_$r.log "$v" "$r" "$OPS" >> gpurun_out/iuab.log <<'PY'
import json, sys
s = open(sys.argv[1]).read(); i = s.find('{"metric"'); d = json.loads(s[i:s.find('\n', i)])
b = d["step_breakdown_ms"]
print(f"r{sys.argv[3]} {sys.argv[2]:6s} {d['ms_per_step']:.3f} ms/step", " ".join(f"{k} {b.get(k, 0):.4f}" for k in sys.argv[4].split()))
PY
  done
done
cat gpurun_out/iuab.log
