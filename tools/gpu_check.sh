#!/bin/bash
# One GPU-box session: parity tests -> smoke -> short bench.  Stops at the first GPU-side
# failure (fault / abort / timeout); an ordinary test assertion failure (rc 1) continues.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout=600 ${PYTEST_ARGS:-} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit 0; fi
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 --breakdown \
  > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -12 gpurun_out/bench.log
exit $rc
