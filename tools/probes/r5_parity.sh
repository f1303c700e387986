#!/bin/bash
# round 5: the headline-size step against the oracle, the unit-gain pair-pass oracle test
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "config1_full_size_step_vs_oracle" > gpurun_out/r5_parity.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r5_parity.log | tail -20; exit $rc
