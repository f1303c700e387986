#!/bin/bash
# one SQ counter pass (8 counters) over the dominant kernel; KERNEL=x6 selects the split-bf16 one
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_sq
tag=${1:-fp32}
out=${2:-$tag}   # second pass: CTRS="..." (at most 8 SQ counters) and another output name
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
KERNEL=$tag timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace \
  --output-format csv -d gpurun_out/pmc_sq/$out -o run -- python3 tools/dominant_kernel.py \
  > gpurun_out/pmc_sq/$out.log 2>&1
rc=$?; echo "pmc $tag rc=$rc"
python3 - "$out" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/pmc_sq/{tag}/**/*counter_collection.csv", recursive=True)
if not f: print("no csv"); sys.exit(0)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if "k_" in r["Kernel_Name"] and "pack" not in r["Kernel_Name"]:
        acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:40s} {c:28s} {sum(v)/len(v):.4g}")
PY
exit $rc
