#!/bin/bash
# bf16x6 kernels: op-level tests, error diagnostics, whole-network x6 parity, N2N bench + profile
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_x6.log 2>&1
rc=$?; echo "x6 op tests rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_x6.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/pytest_x6.log | head -40; exit $rc; fi
timeout -k 10 300 python -u tools/diag_x6.py > gpurun_out/diag_x6.log 2>&1
rc=$?; echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/diag_x6.log | head -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --conv-precision fp32_x6 > gpurun_out/bench_x6.log 2>&1
rc=$?; echo "bench x6 rc=$rc"; tail -c 1200 gpurun_out/bench_x6.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "fp32_x6" --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_x6_net.log 2>&1
rc=$?; echo "x6 net tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_x6_net.log | tail -20
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/pytest_x6_net.log | head -20; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_x6 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline --conv-precision fp32_x6 > $GRAFT_REPO_ROOT/gpurun_out/prof_x6.log 2>&1
echo "rocprof rc=$?"
