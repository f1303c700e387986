"""Does the HIP training path actually learn to denoise?  (VERDICT r1 "what's weak" #10: the
bench's eval leg after ~20 steps only proves HIP == oracle, not denoising.)

Trains the bench workload (N2N step, UNet(48), 64 x 1 x 256^2 per step, Adam lr 3e-4, gauss25;
train.py:330-368 / training_script.md:128-155) from the reference initialisation on fresh
synthetic clean batches (bench.synthetic_clean: smooth random fields), and at checkpoints
denoises the bench's 512^2 eval image (evaluation.py:66-108 on the HIP path), printing its PSNR
next to the noisy input's.  At the end the same weights go through the CPU oracle restatement of
the reference's evaluation (test infrastructure, as in bench.py's cpu_baseline leg) so the
reported PSNR is also the reference's.

    python tools/convergence.py [--steps 600] [--every 100] [--bs 64] [--size 256]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from image_denoising_amd import UNet  # noqa: E402
from image_denoising_amd.trainer import N2NTrainer  # noqa: E402


def noisy_psnr(clean8, noisy8):
    d = clean8.astype(np.float64) - noisy8.astype(np.float64)
    return float(10 * np.log10(255.0 ** 2 / np.mean(d * d)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--bs", type=int, default=64)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "convergence.json"))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = UNet(in_nc=1, out_nc=1, n_feature=48).to(dev).set_precision("fp32_x6")
    tr = N2NTrainer(net, lr=3e-4, n_epoch=100)
    clean8, noisy8 = bench.eval_image()
    rec = {"workload": f"N2N UNet(48) {args.bs}x1x{args.size}^2 per step, Adam 3e-4, gauss25, "
                       "synthetic smooth fields; eval: 512^2 synthetic image",
           "noisy_psnr": round(noisy_psnr(clean8, noisy8), 4), "points": []}
    t0 = time.time()
    for step in range(args.steps + 1):
        if step % args.every == 0:
            torch.cuda.synchronize()
            ps, ss = bench.hip_eval(net, clean8, noisy8)
            p = {"step": step, "psnr": round(ps, 4), "ssim": round(ss, 5),
                 "seconds": round(time.time() - t0, 1)}
            rec["points"].append(p)
            print(json.dumps(p), flush=True)
        if step == args.steps:
            break
        clean = bench.synthetic_clean(args.bs, args.size, args.size, 1000 + step, dev)
        tr.train_step(clean, epoch=1)
    torch.cuda.synchronize()
    ref = bench.oracle_eval_psnr(net.flat_params, clean8, noisy8)
    rec["final_psnr_oracle"] = round(ref, 4)
    rec["final_psnr_abs_diff"] = round(abs(ref - rec["points"][-1]["psnr"]), 6)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "points"}), flush=True)


if __name__ == "__main__":
    main()
