#!/bin/bash
# round 5: deconv full-line stores -- deconv parity tests, then the step's FETCH / WRITE PMC
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6.py tests/test_gpu_parity.py -m gpu -x -q -k "deconv or n2n_step_vs or config1_full_size_step_props" --timeout 240 --timeout-method thread > gpurun_out/deconv_tests.log 2>&1 || { grep -E "FAILED|assert|Error" gpurun_out/deconv_tests.log | head -20; exit 3; }
tail -1 gpurun_out/deconv_tests.log
bash tools/gpu_run.sh pmc:r5b quick || exit 4
