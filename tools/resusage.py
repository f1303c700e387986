"""Per-kernel VGPR / spill / LDS report of one csrc file for gfx950:
    python tools/resusage.py conv_w6.hip [name-regex]"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "image_denoising_amd", "csrc")
src, flt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else ".")
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fno-slp-vectorize", "-x", "hip",
       "-c", os.path.join(CSRC, src), "-o", "/tmp/resusage.o", f"-I{CSRC}", f"-I{os.path.join(CSRC, '..', '..', 'include')}",
       *os.environ.get("DN_EXTRA_CXXFLAGS", "").split(), "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark:\s*([^:]+): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if re.search(flt, r["name"]):
        g = lambda k: r.get(k, "?")
        print(f"{g('VGPRs'):>4} vgpr {g('AGPRs'):>3} agpr spill {g('VGPRs Spill'):>4} lds {g('LDS Size [bytes/block]'):>6} "
              f"occ {g('Occupancy [waves/SIMD]')}  {r['name'][:110]}")
