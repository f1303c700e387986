#!/bin/bash
# round 6: correctness of the changed kernels, then a same-box library A/B (tools/probes/r5_libab.sh)
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_x6.py} -m gpu -x -q --timeout 240 --timeout-method thread ${TK:+-k "$TK"} > gpurun_out/r6_ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6_ab_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|^E " gpurun_out/r6_ab_tests.log | head -20; exit $rc; }
bash tools/probes/r5_libab.sh
