#!/bin/bash
# step-level A/B of environment settings: VARS = space-separated 'NAME=VALUE' (or '-' for none),
# ROUNDS rounds each; per run ms/step and the breakdown entries named in OPS
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
VARS=${VARS:-"- DN_C1S_ALIGN=32"}; OPS=${OPS:-"fwd3 wgrad3 dgrad3 deconv wgrad_up deconv_dgrad"}
: > gpurun_out/envab.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARS; do
    if [ "$v" = "-" ]; then e=""; else e="$v"; fi
    env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eval > gpurun_out/envab_${r}_${v//[=\/]/_}.log 2>&1 || exit $?
    python3 - gpurun_out/envab_${r}_${v//[=\/]/_}.log "$v" "$r" "$OPS" >> gpurun_out/envab.log <<'PY'
import json, sys
s = open(sys.argv[1]).read(); i = s.find('{"metric"'); d = json.loads(s[i:s.find('\n', i)])
b = d["step_breakdown_ms"]
print(f"r{sys.argv[3]} {sys.argv[2]:18s} {d['ms_per_step']:.3f} ms/step", " ".join(f"{k} {b.get(k, 0):.4f}" for k in sys.argv[4].split()))
PY
  done
done
cat gpurun_out/envab.log
