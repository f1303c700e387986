#!/bin/bash
# HBM traffic of the dominant kernel: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes
# (KERNEL=x6: the split-bf16 fp32 kernel of --conv-precision fp32_x6)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc/$c -o run \
    -- python3 tools/dominant_kernel.py > gpurun_out/pmc/$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
find gpurun_out/pmc -name '*.csv' | head
