#!/bin/bash
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python -u tools/probes/r5_wg16.py > gpurun_out/wg16.log 2>&1 || exit $?
cat gpurun_out/wg16.log
rm -rf gpurun_out/prof_wg16
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wg16 -o run -- python3 tools/probes/r5_wg16.py > gpurun_out/prof_wg16.log 2>&1 || exit $?
f=$(find gpurun_out/prof_wg16 -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 $f | head -30
