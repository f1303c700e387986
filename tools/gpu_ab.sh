#!/bin/bash
# A/B of bench configurations: each argument is "ENV=VAL ... -- bench args"
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i+1))
  envs="${spec%%--*}"; args="${spec#*--}"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline $args > gpurun_out/ab_$i.log 2>&1
  rc=$?
  python3 - "$i" "$spec" <<'PY'
import json, sys
i, spec = sys.argv[1], sys.argv[2]
for l in open(f"gpurun_out/ab_{i}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        r = d["roofline"]
        print(f"[{spec}] {d['value']} patches/s  {d['ms_per_step']} ms/step  kernel {r['achieved']} TF/s ({r['avg_launch_ms']} ms)")
PY
  [ $rc -ne 0 ] && { echo "rc=$rc for $spec"; tail -5 gpurun_out/ab_$i.log; exit $rc; }
done
exit 0
