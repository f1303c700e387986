#!/bin/bash
# same-library A/B of run-time switches: SPECS = "name=ENV=VAL[,ENV=VAL] ..." ('-' for none), ROUNDS
# rounds each; per run the bench line's ms/step, the breakdown entries in OPS and the per-shape
# launch times of the kernels matching KSEL (substring)
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -q --timeout 240 --timeout-method thread ${TK:+-k "$TK"} > gpurun_out/r6_envab_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/r6_envab_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E " gpurun_out/r6_envab_tests.log | head -20; exit $rc; }
fi
: > gpurun_out/envab.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in $SPECS; do
    name=${spec%%=*}; envs=${spec#*=}; [ "$envs" = "-" ] && envs=""
    env ${envs//,/ } timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eval ${BARGS:-} > gpurun_out/envab_${name}_$r.log 2>&1 || exit $?
    python3 - gpurun_out/envab_${name}_$r.log "$name" "$r" "${OPS:-}" "${KSEL:-}" >> gpurun_out/envab.log <<'PY'
import json, sys
s = open(sys.argv[1]).read(); i = s.find('{"metric"'); d = json.loads(s[i:s.find('\n', i)])
b = d["step_breakdown_ms"]
ks = [x for x in d["roofline"]["per_shape"] if sys.argv[5] and sys.argv[5] in x["kernel"]]
print(f"r{sys.argv[3]} {sys.argv[2]:8s} {d['ms_per_step']:.3f} ms/step", " ".join(f"{k} {b.get(k, 0):.4f}" for k in sys.argv[4].split()),
      " | ".join(f"{x['kernel']} {x['shape'].split(' ')[0]}@{x['shape'].split('x')[-1]} {x['avg_launch_ms']:.4f}" for x in ks[:6]))
PY
  done
done
cat gpurun_out/envab.log
