#!/bin/bash
# full GPU suite + graft smoke on the committed tree
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_final.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_final.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
