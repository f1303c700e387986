#!/bin/bash
# One parameterised GPU driver for the box (replaces round 2's one-off gpu_r2*.sh probes):
#   bash tools/gpu_run.sh STEP [STEP ...]      steps run in order, each under its own timeout,
#                                              the first failure ends the call (no retries)
# STEP: tests[:FILES]   pytest -m gpu (all, or comma-separated files)  -> gpurun_out/pytest_gpu.log
#       bench           default bench line, CPU baseline included      -> gpurun_out/bench.log
#       quick[:ARGS]    bench line without the CPU baseline ('+'-separated bench args) -> gpurun_out/quick.log
#       stats:TAG[:ARGS] rocprofv3 --kernel-trace --stats over a 3-step bench ('+'-separated bench
#                       args) -> gpurun_out/prof/TAG, plus the step timeline
#       pmc:TAG[:ARGS]  FETCH_SIZE / WRITE_SIZE passes over a 2-step bench -> profiles/TAG_pmc_step.json
#       stamps:TAG:K+N+H  k_c3x6p stage timeline from a DN_X6_STAMPS build (tools/x6_stamps.py)
#       sq:NAME:CTRS    one SQ counter pass (<= 8 SQ counters, '+'-separated) over a 2-step bench
#       micro           tools/x6_micro.py (isolated 3x3 shapes)         -> gpurun_out/micro.log
#       torchrun1       torchrun --nproc-per-node 1 bench (a one-rank RCCL group) -> gpurun_out/torchrun1.log
#       configs         tools/gpu_configs.sh (secondary configurations)
#       smoke           __graft_entry__ build + smoke
#       ab:LIBS         x6_micro per variant library (comma-separated DN_BUILD_TAGs; '-' = default)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
fail() { echo "step '$1' failed (rc=$2)"; exit "$2"; }
summ_stats() {
  local f
  f=$(find "$1" -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms")
for r in rows[:22]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {float(r["Percentage"]):6.2f}% n={r["Calls"]:>5} avg={float(r["AverageNs"])/1e3:9.1f}us  {r["Name"][:100]}')
PY
}
for step in "$@"; do
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "== $step"
  case $name in
    tests)
      files=${arg//,/ }; files=${files:-tests}
      timeout -k 10 1000 python -u -m pytest $files -m gpu -x -v --timeout 240 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
      [ $rc -ne 0 ] && { grep -E "FAILED|^E " gpurun_out/pytest_gpu.log | head -30; fail "$step" $rc; } ;;
    bench)
      timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || fail "$step" $?
      grep '^{' gpurun_out/bench.log | cut -c1-400 ;;
    quick)
      timeout -k 10 240 python -u bench.py --no-cpu-baseline ${arg//+/ } > gpurun_out/quick.log 2>&1 || fail "$step" $?
      grep '^{' gpurun_out/quick.log | cut -c1-400 ;;
    stats)  # stats:TAG[:bench args, '+'-separated]
      tag=${arg%%:*}; bargs=${arg#*:}; [ "$bargs" = "$arg" ] && bargs=""; bargs=${bargs//+/ }
      rm -rf gpurun_out/prof/$tag; mkdir -p gpurun_out/prof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$tag -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $bargs > gpurun_out/prof/$tag.log 2>&1 || fail "$step" $?
      summ_stats gpurun_out/prof/$tag
      f=$(find gpurun_out/prof/$tag -name '*kernel_trace.csv' | head -1)
      [ -n "$f" ] && python3 tools/step_timeline.py "$f" ;;
    pmc)  # pmc:TAG[:bench args, '+'-separated]
      tag=${arg%%:*}; bargs=${arg#*:}; [ "$bargs" = "$arg" ] && bargs=""; bargs=${bargs//+/ }
      rm -rf gpurun_out/pmc_step_$tag; mkdir -p gpurun_out/pmc_step_$tag
      for c in FETCH_SIZE WRITE_SIZE; do
        DN_STEP_STREAMS=0 timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_step_$tag/$c -o run \
          -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-eval $bargs > gpurun_out/pmc_step_$tag/$c.log 2>&1 || fail "$step $c" $?
      done
      python3 tools/pmc_step.py $tag gpurun_out/pmc_step_$tag || fail "$step summary" $? ;;
    stamps)  # stamps:TAG:K+NOUT+H (a DN_X6_STAMPS=1 build libdenoise_hip_TAG.so, tools/x6_stamps.py)
      tag=${arg%%:*}; shp=${arg#*:}
      DN_LIB_PATH=image_denoising_amd/libdenoise_hip_$tag.so timeout -k 10 120 python -u tools/x6_stamps.py ${shp//+/ } \
        > gpurun_out/stamps_${tag}_${shp//+/_}.log 2>&1 || fail "$step" $?
      sed "s/^/$tag: /" gpurun_out/stamps_${tag}_${shp//+/_}.log | grep -v amdgpu.ids ;;
    sq)
      out=${arg%%:*}; ctrs=${arg#*:}; ctrs=${ctrs//+/ }
      rm -rf gpurun_out/pmc_sq/$out; mkdir -p gpurun_out/pmc_sq/$out
      timeout -s KILL 200 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/pmc_sq/$out -o run \
        -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${SQ_ARGS:-} > gpurun_out/pmc_sq/$out.log 2>&1 || fail "$step" $?
      # (SQ_ARGS: extra bench arguments, e.g. SQ_ARGS="--mode finetune --precision bf16")
      python3 tools/pmc_sq_summary.py gpurun_out/pmc_sq/$out ;;
    micro)
      timeout -k 10 300 python -u tools/x6_micro.py > gpurun_out/micro.log 2>&1 || fail "$step" $?
      cat gpurun_out/micro.log ;;
    torchrun1)
      timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --no-cpu-baseline \
        > gpurun_out/torchrun1.log 2>&1 || fail "$step" $?
      grep '^{' gpurun_out/torchrun1.log | cut -c1-600 ;;
    configs)
      timeout -k 10 1200 bash tools/gpu_configs.sh || fail "$step" $? ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1 || fail "$step" $?
      tail -2 gpurun_out/smoke.log ;;
    ab)
      for r in 1 2; do
        for v in ${arg//,/ }; do
          if [ "$v" = "-" ]; then lib=image_denoising_amd/libdenoise_hip.so; else lib=image_denoising_amd/libdenoise_hip_$v.so; fi
          DN_LIB_PATH=$lib timeout -k 10 240 python -u tools/x6_micro.py > gpurun_out/ab_${v}_$r.log 2>&1 || fail "$step $v" $?
          sed "s/^/r$r $v: /" gpurun_out/ab_${v}_$r.log
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
