#!/bin/bash
# training-convergence check of the bench workload (tools/convergence.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/convergence.py --steps ${STEPS:-1500} --every ${EVERY:-250} > gpurun_out/convergence.log 2>&1
rc=$?; cat gpurun_out/convergence.log | grep -v amdgpu.ids; exit $rc
