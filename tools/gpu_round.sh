#!/bin/bash
# full GPU test suite, default bench, rocprof kernel stats of the default bench, PMC traffic (x6)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_default.log | cut -c1-600
[ $rc -ne 0 ] && { tail -5 gpurun_out/bench_default.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_default -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_default.log 2>&1
rc=$?; echo "rocprof rc=$rc"
cd $GRAFT_REPO_ROOT
db=$(find gpurun_out/prof_default -name '*.db' | head -1)
[ -n "$db" ] && python3 tools/kstats.py "$db" --csv gpurun_out/prof_default_kernel_stats.csv --top 40
[ $rc -ne 0 ] && exit $rc
[ "${SKIP_PMC:-0}" = "1" ] && exit 0
KERNEL=x6 bash tools/pmc.sh && python3 tools/pmc_summary.py ${TAG:-r2} x6
