#!/bin/bash
# quick kernel iteration: probes, x6 micro timings, the x6 + parity GPU tests, the bench (tag = $1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-iter}
if [ -x tools/probes/mfma_pattern ]; then timeout -k 10 60 ./tools/probes/mfma_pattern || exit 1; fi
timeout -k 10 180 python -u tools/x6_micro.py > gpurun_out/micro_$TAG.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_x6.py tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_$TAG.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_$TAG.log | cut -c1-300
exit $rc
