set -o pipefail
mkdir -p gpurun_out/mt3
B="python bench.py --mode finetune --precision bf16 --steps 30 --warmup 5"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mt3/tests_bf16.log 2>&1 &&
timeout -k 10 150 $B > gpurun_out/mt3/b_default_1.log 2>&1 &&
DN_BF16_MT3=4 timeout -k 10 150 $B > gpurun_out/mt3/b_mt34_1.log 2>&1 &&
timeout -k 10 150 $B > gpurun_out/mt3/b_default_2.log 2>&1 &&
DN_BF16_MT3=4 timeout -k 10 150 $B > gpurun_out/mt3/b_mt34_2.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/mt3/b_n2n.log 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mt3/pytest_gpu.log 2>&1
