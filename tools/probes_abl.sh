cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/probes/mfma_pattern || exit 1
echo "persistent"; DN_X6_PERSIST=1 timeout -k 10 120 python -u tools/x6_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "old"; timeout -k 10 120 python -u tools/x6_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
DN_X6_PERSIST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_x6.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
