#!/bin/bash
# round-end evidence: full GPU suite + default bench + rocprof + PMC (gpu_round.sh), then the
# secondary configuration bench lines (gpu_configs.sh)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_round.sh || exit $?
bash tools/gpu_configs.sh
