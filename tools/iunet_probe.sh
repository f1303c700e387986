#!/bin/bash
# ImprovedUNet N2N step: bench for each DN_NT2_MT value, plus a kernel-stats profile of the default
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for mt in 4 8 12; do
  DN_NT2_MT=$mt timeout -k 10 300 python bench.py --arch UNetImproved --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/iu_mt$mt.log 2>&1 || exit 1
  echo "MT=$mt $(tail -1 gpurun_out/iu_mt$mt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
