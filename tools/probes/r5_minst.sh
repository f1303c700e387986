#!/bin/bash
# A/B: minimum 32-pixel stages per weight-gradient split (slab bytes vs parallelism)
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
: > gpurun_out/minst.log
for m in 0 4 8 16 0 8; do
  echo "== DN_WG_MINST=$m" >> gpurun_out/minst.log
  DN_WG_MINST=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/minst_$m.log 2>&1 || exit $?
  python3 - gpurun_out/minst_$m.log >> gpurun_out/minst.log <<'PY'
import json, sys
s = open(sys.argv[1]).read(); i = s.find('{"metric"'); d = json.loads(s[i:s.find('\n', i)])
b = d["step_breakdown_ms"]
print(d["ms_per_step"], "wgrad3", b["wgrad3"], "reduce", b["reduce"], "wgrad1", b.get("wgrad1"), "wgrad_up", b.get("wgrad_up"))
for p in d["roofline"]["per_shape"]:
    if p["op"] == "wgrad3": print("   ", p["shape"], p["avg_launch_ms"])
PY
done
cat gpurun_out/minst.log
