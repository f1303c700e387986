#!/bin/bash
# adapter finetune: GPU tests + configs[4] bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_adapter.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_adapter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_adapter.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --mode finetune --steps 10 --warmup 2 > gpurun_out/bench_ft.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_ft.log
exit $rc
