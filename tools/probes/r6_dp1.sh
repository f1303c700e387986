#!/bin/bash
# one-GPU cost of the data-parallel path: plain bench vs a one-rank torchrun group with the
# overlapped two-bucket all-reduce (DN_AR_OVERLAP=1, default) and with one all-reduce after the
# backward (DN_AR_OVERLAP=0); two alternating rounds
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
: > gpurun_out/dp1.log
ms() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"])'; }
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eval > gpurun_out/dp1_plain_$r.log 2>&1 || exit $?
  echo "r$r plain $(ms gpurun_out/dp1_plain_$r.log)" >> gpurun_out/dp1.log
  for ov in ${OVS:-1 0}; do
    DN_AR_OVERLAP=$ov timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --no-cpu-baseline --no-eval \
      > gpurun_out/dp1_ov${ov}_$r.log 2>&1 || exit $?
    echo "r$r torchrun overlap=$ov $(ms gpurun_out/dp1_ov${ov}_$r.log)" >> gpurun_out/dp1.log
  done
done
cat gpurun_out/dp1.log
