#!/bin/bash
# step-level A/B of variant libraries: LIBS = tags ('-' = the default build), two rounds each;
# per run the bench line's ms/step and the step breakdown entries named in OPS
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
LIBS=${LIBS:-"- base"}; OPS=${OPS:-"wgrad_up wgrad1"}
: > gpurun_out/libab.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $LIBS; do
    if [ "$v" = "-" ]; then lib=image_denoising_amd/libdenoise_hip.so; else lib=image_denoising_amd/libdenoise_hip_$v.so; fi
    DN_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eval ${BARGS:-} > gpurun_out/libab_${v}_$r.log 2>&1 || exit $?
    python3 - gpurun_out/libab_${v}_$r.log "$v" "$r" "$OPS" >> gpurun_out/libab.log <<'PY'
import json, sys
s = open(sys.argv[1]).read(); i = s.find('{"metric"'); d = json.loads(s[i:s.find('\n', i)])
b = d["step_breakdown_ms"]
print(f"r{sys.argv[3]} {sys.argv[2]:6s} {d['ms_per_step']:.3f} ms/step", " ".join(f"{k} {b.get(k, 0):.4f}" for k in sys.argv[4].split()))
PY
  done
done
cat gpurun_out/libab.log
