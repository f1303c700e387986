#!/bin/bash
# hardware-queue sharing: a one-rank torchrun group (RCCL streams + the step's four) with HIP's
# default 4 hardware queues per process vs 8, and the plain bench with 4 vs 8; two rounds
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
: > gpurun_out/hwq.log
ms() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"])'; }
for r in 1 2; do
  for q in ${QS:-4 8}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eval > gpurun_out/hwq_plain_${q}_$r.log 2>&1 || exit $?
    echo "r$r plain q=$q $(ms gpurun_out/hwq_plain_${q}_$r.log)" >> gpurun_out/hwq.log
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --no-cpu-baseline --no-eval \
      > gpurun_out/hwq_tr_${q}_$r.log 2>&1 || exit $?
    echo "r$r torchrun q=$q $(ms gpurun_out/hwq_tr_${q}_$r.log)" >> gpurun_out/hwq.log
  done
done
cat gpurun_out/hwq.log
