#!/bin/bash
# x6 op tests + the 96/144-channel shapes of tools/x6_shapes.py (quick A/B of a kernel change)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_x6.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_x6.log; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/pytest_x6.log | head; exit $rc; }
timeout -k 10 300 python -u tools/x6_shapes.py > gpurun_out/x6_shapes.log 2>&1; rc=$?
grep -E "96 H" gpurun_out/x6_shapes.log; exit $rc
