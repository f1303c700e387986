cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for mt in 4 2 1; do DN_C1_MT=$mt timeout -k 10 200 python - <<'PY' >> gpurun_out/probe.log 2>&1 || exit 1
import os, sys
sys.path.insert(0, ".")
from tools.bench_ops import deconv, conv
print("MT", os.environ["DN_C1_MT"])
deconv(64, 128, 128, 96, 100)
deconv(64, 64, 64, 96, 144)
conv(64, 256, 256, 96, 96, 1, 96, 96)
PY
done
cat gpurun_out/probe.log
