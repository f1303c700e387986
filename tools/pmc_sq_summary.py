"""Per-kernel means of one rocprofv3 SQ counter pass (tools/gpu_run.sh sq:...), with the wait
fractions of MI355X_MICROARCH.md §rocprofv3 (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES):
    python tools/pmc_sq_summary.py gpurun_out/pmc_sq/NAME"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
if not f:
    sys.exit(f"no counter CSV under {d}")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)  # kernel -> dispatch -> ns
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dn::", "").replace(" ", "")
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[k][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
rows = sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0])))
for k, cs in rows[:24]:
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    line = f"{k[:44]:44s} n={len(next(iter(cs.values()))):3d}"
    wc = m.get("SQ_WAVE_CYCLES")
    for c, v in sorted(m.items()):
        line += f"  {c.replace('SQ_', '')}={v:.4g}"
        if wc and c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            line += f"({v / wc:.3f})"
    # MFMA pipe utilisation: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs) over the
    # 1024 SIMDs x the dispatch's shader cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs);
    # effective clock = GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS give-back)
    ga = m.get("GRBM_GUI_ACTIVE")
    if ga and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        line += f"  mfma_util={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (ga / 8 * 1024):.3f}"
    ns = sum(dur[k].values()) / max(1, len(dur[k]))
    if ga and ns > 0:
        line += f"  clock_GHz={ga / 8 / ns:.2f}  mean_ns={ns:.0f}"
    print(line)
