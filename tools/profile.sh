#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run -> gpurun_out/prof/<tag>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-bench}
shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run \
  -- python3 bench.py --steps ${PROF_STEPS:-3} --warmup 1 --no-cpu-baseline "$@" > gpurun_out/prof/$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"
f=$(find gpurun_out/prof/$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms")
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {float(r["Percentage"]):6.2f}% n={r["Calls"]:>5} avg={float(r["AverageNs"])/1e3:9.1f}us  {r["Name"][:110]}')
PY
exit $rc
