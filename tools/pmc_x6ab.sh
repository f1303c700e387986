#!/bin/bash
# SQ counters of the dominant x6 shape, persistent kernel vs the per-tile one (A/B)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_ab
CTRS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS"
for v in q p; do
  if [ $v = q ]; then export DN_X6_PERSIST=1; else unset DN_X6_PERSIST; fi
  KERNEL=x6 REPS=3 timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
    -d gpurun_out/pmc_ab/$v -o run -- python3 tools/dominant_kernel.py > gpurun_out/pmc_ab/$v.log 2>&1
  echo "pmc $v rc=$?"
done
python3 - <<'PY'
import csv, glob, collections
for v in ("q", "p"):
    f = glob.glob(f"gpurun_out/pmc_ab/{v}/**/*counter_collection.csv", recursive=True)
    if not f: print(v, "no csv"); continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "k_c3x6" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    wc = sum(acc["SQ_WAVE_CYCLES"]) / len(acc["SQ_WAVE_CYCLES"])
    print(v, " ".join(f"{k}={sum(x)/len(x):.4g}" for k, x in sorted(acc.items())))
    print(v, "fractions of wave cycles:", {k: round(sum(acc[k]) / len(acc[k]) / wc, 3) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")})
PY
