#!/bin/bash
# round 5: k_wgrad3q with conflict-free write slots -- weight tests, isolated A/B against
# libdenoise_hip_base.so, then the SQ pass of the bench step
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6.py tests/test_gpu_parity.py -m gpu -x -q -k "weight or unit_gain" --timeout 300 --timeout-method thread > gpurun_out/wq_tests.log 2>&1 || { grep -E "FAILED|assert|Error" gpurun_out/wq_tests.log | head -20; exit 3; }
tail -1 gpurun_out/wq_tests.log
for r in 1 2 3; do for v in base -; do
  lib=image_denoising_amd/libdenoise_hip.so; [ "$v" = "-" ] || lib=image_denoising_amd/libdenoise_hip_$v.so
  DN_LIB_PATH=$lib timeout -k 10 200 python -u - > gpurun_out/wq_${v}_$r.log 2>&1 <<'PY' || { tail -5 gpurun_out/wq_${v}_$r.log; exit 4; }
import os, sys
sys.path.insert(0, os.getcwd())
from tools.x6_shapes import wgrad
ms = wgrad(48, 48, 128, True)
fl = 2.0 * 64 * 128 * 128 * 48 * 48 * 9
print(f"48->48@128 {ms:.3f}ms/{fl / ms / 1e9 / (2500 / 6):.3f}")
PY
  sed "s/^/r$r $v: /" gpurun_out/wq_${v}_$r.log | grep -v amdgpu.ids
done; done
bash tools/gpu_run.sh sq:r5q:SQ_ACTIVE_INST_ANY+SQ_LDS_BANK_CONFLICT+SQ_LDS_IDX_ACTIVE+SQ_VALU_MFMA_BUSY_CYCLES+SQ_WAIT_ANY+SQ_WAIT_INST_ANY+SQ_INSTS_VALU+SQ_WAVE_CYCLES+GRBM_GUI_ACTIVE > gpurun_out/wq_sq.log 2>&1 || exit 5
grep wgrad3 gpurun_out/wq_sq.log | cut -c1-300
