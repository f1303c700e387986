"""Summarise tools/pmc.sh output into profiles/<tag>_pmc_dominant.json (read by bench.py).
Corrections per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reports half the bytes of a 16-B-per-lane streaming read, so reads are doubled."""
import csv
import json
import os
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
kind = sys.argv[2] if len(sys.argv) > 2 else ""  # x6 / bf16 (KERNEL=... tools/pmc.sh)
x6 = kind == "x6"
kname = {"x6": "k_c3x6", "bf16": "k_fwd_bf16"}.get(kind, "k_fwd<")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = list(csv.DictReader(open(os.path.join(root, "gpurun_out/pmc", c, "run_counter_collection.csv"))))
    v = [float(r["Counter_Value"]) for r in rows if kname in r["Kernel_Name"] and r["Counter_Name"] == c]
    vals[c] = v
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"]) * 1024 * 2
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) * 1024
bs, H, W, C = (16, 512, 512, 96) if kind == "bf16" else (64, 256, 256, 96)
alg = bs * H * W * C * 4 * 2 + 96 * 96 * 9 * 4
out = {"kernel": {"x6": "k_c3x6p<NT=6> (bf16x6 split fp32)", "bf16": "k_fwd_bf16p<6,4> (bf16 base)"}
                 .get(kind, "k_fwd<G_C3,NT=6,MT=4>") + f" dec_conv1b-shaped 96->96 3x3, {bs}x{H}x{W}",
       "launches": len(vals["FETCH_SIZE"]), "fetch_bytes_corrected": fetch, "write_bytes": write,
       "traffic_bytes": fetch + write, "algorithmic_bytes": alg,
       "traffic_over_algorithmic": (fetch + write) / alg,
       "raw_FETCH_SIZE_KiB": vals["FETCH_SIZE"], "raw_WRITE_SIZE_KiB": vals["WRITE_SIZE"],
       "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes with "
                 "--kernel-trace (tools/pmc.sh); FETCH x2 gfx950 correction"}
name = f"{tag}_pmc_dominant_{kind}.json" if kind else f"{tag}_pmc_dominant.json"
json.dump(out, open(os.path.join(root, "profiles", name), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if not k.startswith("raw")}, indent=1))
