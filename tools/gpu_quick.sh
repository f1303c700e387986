#!/bin/bash
# GPU tests, default bench, rocprof kernel stats of a short bench run (tag = $1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-quick}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_$TAG.log | cut -c1-330
[ $rc -ne 0 ] && { tail -5 gpurun_out/bench_$TAG.log; exit $rc; }
bash tools/profile.sh $TAG
