#!/bin/bash
# roofline evidence: PMC HBM traffic (x6 dominant kernel, bf16 base kernel), SQ counters of the
# x6 kernel, and the configs[4] bf16 finetune bench + its kernel stats (tag = $1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r2}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
KERNEL=x6 bash tools/pmc.sh && python3 tools/pmc_summary.py $TAG x6 > gpurun_out/pmc_x6_summary.txt || exit 1
rm -rf gpurun_out/pmc_x6 && mv gpurun_out/pmc gpurun_out/pmc_x6
KERNEL=bf16 bash tools/pmc.sh && python3 tools/pmc_summary.py $TAG bf16 > gpurun_out/pmc_bf16_summary.txt || exit 1
rm -rf gpurun_out/pmc_bf16 && mv gpurun_out/pmc gpurun_out/pmc_bf16
bash tools/pmc_sq.sh x6 > gpurun_out/pmc_sq_x6_summary.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --mode finetune --precision bf16 --no-cpu-baseline > gpurun_out/bench_ft_bf16_$TAG.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_ft_bf16_$TAG.log | cut -c1-400
bash tools/profile.sh ft_bf16_$TAG --mode finetune --precision bf16
cp profiles/${TAG}_pmc_dominant_x6.json profiles/${TAG}_pmc_dominant_bf16.json gpurun_out/ 2>/dev/null
cat gpurun_out/pmc_x6_summary.txt gpurun_out/pmc_bf16_summary.txt gpurun_out/pmc_sq_x6_summary.txt
