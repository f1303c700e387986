#!/bin/bash
# GPU parity tests (all, or the files given) with per-test timeouts; stops on a GPU-side failure
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
FILES=${@:-tests}
timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -60
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/pytest_gpu.log | head -40; fi
exit $rc
