set -o pipefail
mkdir -p gpurun_out/mt
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
T="python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread"
B="python bench.py --mode finetune --precision bf16 --steps 30 --warmup 5"
timeout -k 10 120 python tools/probes/bf16_mt_ident.py gpurun_out/mt/y4.pt > gpurun_out/mt/ident.log 2>&1 &&
DN_BF16_MT=6 timeout -k 10 120 python tools/probes/bf16_mt_ident.py gpurun_out/mt/y6.pt gpurun_out/mt/y4.pt >> gpurun_out/mt/ident.log 2>&1 &&
DN_BF16_MT3=8 timeout -k 10 120 python tools/probes/bf16_mt_ident.py gpurun_out/mt/y8.pt gpurun_out/mt/y4.pt >> gpurun_out/mt/ident.log 2>&1 &&
DN_BF16_MT=6 DN_BF16_MT3=8 timeout -k 10 300 $T > gpurun_out/mt/tests.log 2>&1 &&
for r in 1 2; do
 timeout -k 10 150 $B > gpurun_out/mt/b_base_$r.log 2>&1 &&
 DN_BF16_MT=6 timeout -k 10 150 $B > gpurun_out/mt/b_mt6_$r.log 2>&1 &&
 DN_BF16_MT3=8 timeout -k 10 150 $B > gpurun_out/mt/b_mt38_$r.log 2>&1 &&
 DN_BF16_MT=6 DN_BF16_MT3=8 timeout -k 10 150 $B > gpurun_out/mt/b_both_$r.log 2>&1 || exit 1
done &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
DN_BF16_MT=6 DN_BF16_MT3=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/mt/prof -o both -- python bench.py --mode finetune --precision bf16 --steps 10 --warmup 3 > gpurun_out/mt/prof.log 2>&1
