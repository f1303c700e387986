cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/x6_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
