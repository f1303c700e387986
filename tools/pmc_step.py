"""HBM bytes per launch of every kernel of the bench step, from rocprofv3 --pmc passes over
`bench.py` (FETCH_SIZE and WRITE_SIZE in separate runs, tools/gpu_run.sh pmc):
    python tools/pmc_step.py TAG  ->  profiles/TAG_pmc_step.json   (read by bench.py)
Corrections per MI355X_MICROARCH.md §HBM: the counters are KiB; on gfx950 FETCH_SIZE reports half
the bytes of a 16-B-per-lane streaming read, so reads are doubled.  Kernel names are normalised
to the labels dn_profile_ops records ("k_c3x6p<6,0,true>")."""
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def norm(name: str) -> str:
    n = name.split("(")[0]
    n = re.sub(r"^void\s+", "", n).replace("dn::", "").replace(" ", "")
    return n


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "pmc_step")
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        path = None
        for dp, _, fs in os.walk(os.path.join(src, c)):
            for f in fs:
                if f.endswith("counter_collection.csv"):
                    path = os.path.join(dp, f)
        if path is None:
            raise SystemExit(f"no counter CSV under {src}/{c}")
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != c:
                continue
            k = norm(r["Kernel_Name"])
            per.setdefault(k, {}).setdefault(c, []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, v in per.items():
        if "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
            continue
        f = [x for _, x in sorted(v["FETCH_SIZE"])]
        w = [x for _, x in sorted(v["WRITE_SIZE"])]
        fetch = sum(f) / len(f) * 1024 * 2
        write = sum(w) / len(w) * 1024
        out[k] = {"launches": len(f), "fetch_bytes_corrected": fetch,
                  "write_bytes": write, "traffic_bytes": fetch + write}
        # per launch in dispatch order (the two passes run the same single-stream launch
        # sequence): bench.py picks the dominant shape's launches out of the last step
        if len(f) == len(w):
            out[k]["per_launch_bytes"] = [round(a * 2048 + b * 1024) for a, b in zip(f, w)]
            out[k]["per_launch_fetch"] = [round(a * 2048) for a in f]
            out[k]["per_launch_write"] = [round(b * 1024) for b in w]
    doc = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes with "
                     "--kernel-trace over `bench.py --steps 2 --warmup 1 --no-cpu-baseline` "
                     "(tools/gpu_run.sh pmc); per-launch means over every dispatch of the kernel "
                     "(all its shapes); FETCH x2 gfx950 correction; per_launch_bytes in dispatch order "
                     "(DN_STEP_STREAMS=0: one stream, the launch order of dn_profile_ops)",
           "kernels": dict(sorted(out.items(), key=lambda kv: -kv[1]["traffic_bytes"]))}
    dst = os.path.join(ROOT, "profiles", f"{tag}_pmc_step.json")
    json.dump(doc, open(dst, "w"), indent=1)
    for k, v in list(doc["kernels"].items())[:12]:
        print(f"{k:40s} {v['launches']:4d} launches  {v['traffic_bytes'] / 1e9:8.3f} GB/launch")


if __name__ == "__main__":
    main()
