#!/bin/bash
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u tools/probes/r5_enc6.py > gpurun_out/r5_enc6.log 2>&1; rc=$?
grep -v Warn gpurun_out/r5_enc6.log | tail -12; exit $rc
