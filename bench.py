"""Training throughput of the N2N U-Net step on MI355X (BASELINE.json metric, config 1).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL)

A step = noise synthesis + neighbour sub-sampling + no-grad UNet(256^2) + UNet(128^2) fwd/bwd
+ N2N loss + [RCCL all-reduce of the flat gradient] + Adam, on bs=64 patches per rank of
synthetic 256x256x1 data (weak scaling: global batch = 64 * N).  Prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix = vector, spec
PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
# fp32 by three-way bf16 splitting: 6 bf16 MFMA products per fp32 product
PEAK_X6_TFLOPS = PEAK_BF16_TFLOPS / 6


def conv_flops(h, w, cin, cout, k):
    return 2.0 * h * w * cin * cout * k * k


def unet_fwd_flops(H, W, C=1, nf=48):
    """analytic forward FLOPs of arch_unet.UNet per image (== torch FlopCounter)"""
    f = conv_flops(H, W, C, nf, 3) + conv_flops(H, W, nf, nf, 3)
    for l in range(1, 6):
        f += conv_flops(H >> l, W >> l, nf, nf, 3)
    f += conv_flops(H >> 5, W >> 5, nf, nf, 1) * 4          # up5 deconv (per output pixel group)
    f += 2 * conv_flops(H >> 4, W >> 4, 2 * nf, 2 * nf, 3)
    for l in (3, 2, 1):
        f += conv_flops(H >> (l + 1), W >> (l + 1), 2 * nf, 2 * nf, 1) * 4
        f += conv_flops(H >> l, W >> l, 3 * nf, 2 * nf, 3) + conv_flops(H >> l, W >> l, 2 * nf, 2 * nf, 3)
    f += conv_flops(H >> 1, W >> 1, 2 * nf, 2 * nf, 1) * 4
    f += conv_flops(H, W, 2 * nf + C, 96, 3) + conv_flops(H, W, 96, 96, 3)
    f += 2 * conv_flops(H, W, 96, 96, 1) + conv_flops(H, W, 96, C, 1)
    return f


def iunet_fwd_flops(H, W, C=1, nf=48):
    """analytic forward FLOPs of arch_unet.ImprovedUNet per image (convs only; GroupNorm,
    activations, pooling and PixelShuffle are elementwise)"""
    f = conv_flops(H, W, C, nf, 3) + conv_flops(H, W, nf, 1, 3)  # noise estimator

    def rdb(h, w, ch):
        return sum(conv_flops(h, w, ch + 32 * j, 32, 3) for j in range(4)) + conv_flops(h, w, ch + 128, ch, 1)

    def res(h, w, ch):
        return 2 * conv_flops(h, w, ch, ch, 3)

    c, cin = nf, C + 1
    for i in range(4):
        h, w = H >> i, W >> i
        f += conv_flops(h, w, cin, c, 3) + rdb(h, w, c) + res(h, w, c)
        cin, c = c, 2 * c
    c //= 2
    f += rdb(H >> 4, W >> 4, c) + res(H >> 4, W >> 4, c)
    for k in range(4):
        o = c // 2
        h, w = H >> (3 - k), W >> (3 - k)
        f += conv_flops(h // 2, w // 2, c, 4 * o, 3) + conv_flops(h, w, 3 * o, o, 3)
        f += rdb(h, w, o) + res(h, w, o)
        c = o
    return f + conv_flops(H, W, nf // 2 + C, C, 3)


def synthetic_clean(n, H, W, seed, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    lo = torch.rand(n, 1, H // 8, W // 8, generator=g)
    return F.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False).to(device)


def time_dominant_kernel(bs, H, W, device, reps=5):
    """dec_conv1b-shaped 3x3 conv (96->96 at 256^2, bs images) through the same k_fwd kernel the
    step uses, timed with HIP events on the stream it is launched on."""
    from image_denoising_amd import _lib

    x = torch.randn(bs, H, W, 96, device=device)
    w = torch.randn(96, 96, 3, 3, device=device) * 0.05
    b = torch.zeros(96, device=device)
    y = torch.empty_like(x)
    s = torch.cuda.current_stream(device)
    pk = _lib.scratch(_lib.lib().dn_conv2d_pack_size(96, 96, 3, 0), device)
    run = lambda: _lib.call("dn_conv2d_forward", x.data_ptr(), 96, bs, H, W, 96, w.data_ptr(),
                            b.data_ptr(), 96, 3, 1, y.data_ptr(), 96, pk.data_ptr(), pk.numel(),
                            s.cuda_stream)
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flops = bs * conv_flops(H, W, 96, 96, 3)
    del x, y
    return ms, flops


def time_dominant_kernel_x6(bs, H, W, device, reps=5):
    """the same 96->96 3x3 shape through the split-bf16 fp32 kernel (--conv-precision fp32_x6)"""
    from image_denoising_amd import _lib

    x = torch.randn(bs, H, W, 96, device=device)
    w = torch.randn(96, 96, 3, 3, device=device) * 0.05
    b = torch.zeros(96, device=device)
    y = torch.empty_like(x)
    s = torch.cuda.current_stream(device)
    pk = _lib.scratch(_lib.lib().dn_conv2d_x6_pack_size(96, 96, 0), device)
    run = lambda: _lib.call("dn_conv2d_forward_x6", x.data_ptr(), 96, bs, H, W, 96,
                            w.data_ptr(), b.data_ptr(), 96, 1, y.data_ptr(), 96, pk.data_ptr(),
                            pk.numel(), s.cuda_stream)
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    e1.synchronize()
    del x, y
    return e0.elapsed_time(e1) / reps, bs * conv_flops(H, W, 96, 96, 3)


def time_dominant_kernel_bf16(bs, H, W, device, reps=5):
    """the same 96->96 3x3 shape through the bf16 matrix-core kernel (finetune --precision bf16)"""
    from image_denoising_amd import _lib

    x = torch.randn(bs, H, W, 96, device=device)
    w = torch.randn(96, 96, 3, 3, device=device) * 0.05
    b = torch.zeros(96, device=device)
    y = torch.empty_like(x)
    s = torch.cuda.current_stream(device)
    pk = _lib.scratch(_lib.lib().dn_conv2d_bf16_pack_size(96, 96), device)
    run = lambda: _lib.call("dn_conv2d_forward_bf16", x.data_ptr(), 96, bs, H, W, 96,
                            w.data_ptr(), b.data_ptr(), 96, 1, y.data_ptr(), 96, pk.data_ptr(),
                            pk.numel(), s.cuda_stream)
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    e1.synchronize()
    del x, y
    return e0.elapsed_time(e1) / reps, bs * conv_flops(H, W, 96, 96, 3)


THREE_BY_THREE = ("fwd3", "fwd3sel", "dgrad3", "wgrad3")


def step_profile(step, reps=2):
    """`reps` extra steps after the timed region with every launch recorded (dn_profile_ops:
    HIP events on the launch stream, executors and the step single-stream so each event pair
    brackets one kernel).  Returns (records, reps)."""
    from image_denoising_amd import _lib

    old = os.environ.get("DN_STEP_STREAMS")
    os.environ["DN_STEP_STREAMS"] = "0"
    torch.cuda.synchronize()
    _lib.profile_ops(True)
    try:
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
        recs = _lib.profile_ops_take()
    finally:
        _lib.profile_ops(False)
        if old is None:
            os.environ.pop("DN_STEP_STREAMS", None)
        else:
            os.environ["DN_STEP_STREAMS"] = old
    return recs, reps


def per_shape_roofline(recs, reps, peak):
    """the step's 3x3 launches grouped by (op, K, NOUT, H, W, kernel): launches per step, mean
    HIP-event ms, algorithmic FLOPs per launch (SEL: the pair pixels it computes) and the fraction
    of `peak`; plus the time-weighted fraction over all of them and the per-op step breakdown"""
    groups = {}
    seen = {}  # launches of each kernel so far: a record's position in its kernel's sequence
    per_kernel = {}
    for r in recs:
        per_kernel[r["kernel"]] = per_kernel.get(r["kernel"], 0) + 1
    for r in recs:
        i = seen.get(r["kernel"], 0)
        seen[r["kernel"]] = i + 1
        if r["op"] not in THREE_BY_THREE:
            continue
        k = (r["op"], r["K"], r["NOUT"], r["H"], r["W"], r["N"], r["kernel"])
        g = groups.setdefault(k, [0, 0.0, 0.0, set()])
        g[0] += 1
        g[1] += r["ms"]
        g[2] += r["flops"]
        g[3].add(i % max(1, per_kernel[r["kernel"]] // reps))
    shapes = []
    for (op, K, NO, H, W, N, kern), (n, ms, fl, pos) in groups.items():
        tf = fl / (ms * 1e-3) / 1e12
        # HBM bytes the launch must move: input + output activations (fp32), weights aside
        alg_bytes = N * H * W * (K + NO) * 4.0
        shapes.append({"op": op, "kernel": kern, "shape": f"{K}->{NO} @{N}x{H}x{W}",
                       "launches_per_step": n / reps, "avg_launch_ms": round(ms / n, 4),
                       "flops_per_launch": fl / n, "tflops": round(tf, 2), "frac": round(tf / peak, 4),
                       "ms_per_step": round(ms / reps, 4), "algorithmic_bytes_per_launch": alg_bytes,
                       "alg_gbs": round(alg_bytes / (ms / n * 1e-3) / 1e9, 1),
                       "_positions": sorted(pos), "_kernel_per_step": per_kernel[kern] // reps})
    shapes.sort(key=lambda d: -d["ms_per_step"])
    tot_ms = sum(d["ms_per_step"] for d in shapes)
    tot_fl = sum(d["flops_per_launch"] * d["launches_per_step"] for d in shapes)
    weighted = (tot_fl / (tot_ms * 1e-3) / 1e12 / peak) if tot_ms else None
    by_op = {}
    for r in recs:
        by_op[r["op"]] = by_op.get(r["op"], 0.0) + r["ms"] / reps
    executed = sum(r["flops"] for r in recs) / reps
    return shapes, weighted, tot_ms, {k: round(v, 4) for k, v in sorted(by_op.items(), key=lambda kv: -kv[1])}, executed


def pmc_step_traffic(shape, mode_tag):
    """HBM bytes per launch of the dominant in-step shape, from the committed rocprofv3 PMC
    summaries profiles/<round>_<mode_tag>_pmc_step.json (tools/gpu_run.sh pmc: separate
    FETCH_SIZE / WRITE_SIZE passes over this bench configuration, one stream; gfx950 x2 FETCH
    correction), newest round first.  The shape's launches are picked out of the summary's last
    step by their positions in the kernel's launch sequence (the dn_profile_ops order); a summary
    without per-launch bytes, or whose launch count does not fit, gives the kernel's mean over
    all its shapes.  Returns (bytes, source, "shape" | "kernel mean") or (None, None, None)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{mode_tag}_pmc_step.json")), reverse=True)
    for f in files:
        k = json.load(open(f)).get("kernels", {}).get(shape["kernel"])
        if not k:
            continue
        per, n = k.get("per_launch_bytes"), shape["_kernel_per_step"]
        if per and n and len(per) >= n and max(shape["_positions"]) < n:
            last = per[len(per) - n:]
            sel = [last[i] for i in shape["_positions"]]
            return sum(sel) / len(sel), os.path.relpath(f, ROOT), "shape"
        return k["traffic_bytes"], os.path.relpath(f, ROOT), "kernel mean"
    return None, None, None


def pmc_traffic(tag=""):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (tools/pmc.sh + tools/pmc_summary.py; FETCH_SIZE x2 gfx950 correction), or None."""
    import glob

    pat = f"*_pmc_dominant_{tag}.json" if tag else "*_pmc_dominant.json"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pat)))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d.get("traffic_bytes"), os.path.relpath(files[-1], ROOT)


def host_cpu_info():
    """the host the CPU baseline runs on: nproc, the cores this process may use (affinity mask
    and cgroup CPU quota: on the GPU box os.cpu_count() is the whole machine, not our share),
    the CPU model"""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    info["cgroup_cpus"] = quota
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    return info


def _time_oracle_step(bs, H, reps, budget_s):
    """median wall time of the oracle N2N step (+ Adam) at bs x 1 x H x H: 1 warm-up, then
    `reps` timed steps (fewer if they would overrun budget_s); returns (median_s, n)"""
    import numpy as np

    from image_denoising_amd.arch_unet import reference_init
    from oracle import philox, unet_ref

    torch.manual_seed(0)
    flat = reference_init(1, 1, 48)
    clean = synthetic_clean(bs, H, H, 0, "cpu")
    noisy = clean + (25.0 / 255.0) * torch.from_numpy(
        philox.normal(0, 0, np.arange(clean.numel(), dtype=np.uint64)).reshape(clean.shape)).float()
    rd = philox.rd_idx(1, 1, bs * (H // 2) * (H // 2))
    t0 = time.perf_counter()
    unet_ref.n2n_step(flat, noisy, rd, 0.02)  # warm-up
    t_end = time.perf_counter() + budget_s
    times = []
    while len(times) < reps and (not times or time.perf_counter() + times[-1] < t_end):
        t0 = time.perf_counter()
        unet_ref.n2n_step(flat, noisy, rd, 0.02)
        times.append(time.perf_counter() - t0)
    return sorted(times)[len(times) // 2], len(times)


def cpu_baseline(budget_s=150.0):
    """the oracle (torch-CPU restatement of the reference N2N step +
    Adam, validated against the reference in tests/test_oracle_golden.py) on the host cores of
    the GPU box, at config 0 (8 x 1 x 128^2) and at config 1's shape (64 x 1 x 256^2, the
    workload of `value`); median of 5 after 1 warm-up (config 1: fewer if 5 would overrun the
    budget; the count is reported).  Threads = the cores this process may use."""
    info = host_cpu_info()
    threads = info["affinity"] or 1
    if info["cgroup_cpus"]:
        threads = min(threads, info["cgroup_cpus"])
    torch.set_num_threads(threads)
    t0, n0 = _time_oracle_step(8, 128, 5, budget_s)
    t1, n1 = _time_oracle_step(64, 256, 5, budget_s)
    return {"value": round(64 / t1, 3), "unit": "patches/s", "cores": threads, "kind": "port",
            "sample": f"oracle N2N step (torch-CPU restatement of train.py/arch_unet.py) + Adam at "
                      f"config 1's shape, 64x1x256x256, nf=48; median of {n1} after 1 warm-up",
            "configs": {"config0_8x1x128x128": {"patches_per_s": round(8 / t0, 3),
                                                "s_per_step": round(t0, 4), "timed_steps": n0},
                        "config1_64x1x256x256": {"patches_per_s": round(64 / t1, 3),
                                                 "s_per_step": round(t1, 4), "timed_steps": n1}},
            "host": info, "threads": threads}


def eval_image(seed=11, size=512):
    """one synthetic uint8 image pair for the eval-PSNR leg: smooth clean field, gauss25 noise
    (train.py:84-94 on the [0,255] scale), both clipped to uint8 (evaluation.py reads PNGs)"""
    import numpy as np

    clean = synthetic_clean(1, size, size, seed, "cpu")[0, 0].numpy()
    g = torch.Generator().manual_seed(seed + 1)
    noise = torch.randn(size, size, generator=g).numpy()
    clean8 = np.clip(clean * 255.0 + 0.5, 0, 255).astype(np.uint8)
    noisy8 = np.clip(clean8.astype(np.float32) + 25.0 * noise + 0.5, 0, 255).astype(np.uint8)
    return clean8, noisy8


def hip_eval(net, clean8, noisy8):
    """evaluation.py:66-108 on the HIP path: denoise the full image, PSNR / SSIM on device"""
    from image_denoising_amd.evaluation import evaluate

    r = evaluate(net, [clean8], [noisy8], tiled=False)
    return r["avg_psnr"], r["avg_ssim"]


def oracle_eval_psnr(flat, clean8, noisy8, in_nc=1):
    """the same image through the CPU oracle (torch-CPU restatement of the reference UNet and of
    utils_eval.calculate_psnr) with the same trained weights"""
    import numpy as np

    from oracle import eval_ref, unet_ref

    x = torch.from_numpy(noisy8.astype(np.float32) / 255.0)[None, None]
    with torch.no_grad():
        pred = unet_ref.forward(flat.detach().cpu(), x, in_nc, in_nc)[0, 0].numpy()
    return float(eval_ref.psnr(eval_ref.quantize_full(pred), clean8))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--bs", type=int, default=None, help="patches per GPU (64; finetune: 16)")
    ap.add_argument("--size", type=int, default=None, help="patch edge (256; finetune: 512)")
    ap.add_argument("--channels", type=int, default=1)
    ap.add_argument("--mode", choices=["n2n", "structure", "finetune"], default="n2n",
                    help="n2n: the N2N step (BASELINE metric); structure: train.py's "
                         "Structure_loss step (two grad forwards at full resolution); finetune: "
                         "finetune.py's adapter step (frozen UNet base + OutputAdapter, configs[4])")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                    help="finetune only: bf16 = mixed-precision frozen base (BASELINE configs[4])")
    ap.add_argument("--conv-precision", choices=["fp32", "fp32_x6"], default="fp32_x6",
                    help="UNet 3x3 convs: fp32 operands split exactly into three bf16 pieces on "
                         "the bf16 matrix cores (fp32_x6, default: fp32-accurate, DESIGN.md §12), "
                         "or fp32 operands on the fp32 matrix cores")
    ap.add_argument("--arch", choices=["UNet", "UNetImproved"], default="UNet",
                    help="network (train.py:305-313 / finetune.py --arch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-eval", action="store_true",
                    help="skip the eval-PSNR leg (and the CPU baseline that shares its image): "
                         "under rocprofv3 --pmc the profiled step pair is then the run's last launches")
    ap.add_argument("--breakdown", action="store_true", help="per-phase HIP-event timing (stderr)")
    args = ap.parse_args()

    from image_denoising_amd import dist as dp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DN_DIST_BACKEND=gloo rehearses the multi-process path with every rank on the visible GPUs
    # (round-robin), e.g. 2 ranks on a 1-GPU box; the real runs use RCCL ("nccl"), one GPU each
    backend = os.environ.get("DN_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    # a process group whenever torchrun started us (world 1 included: a one-rank RCCL group runs
    # the same broadcast + per-step all-reduce as N ranks) or world > 1
    os.environ["LOCAL_RANK"] = str(local)
    dp.init_from_env(backend)
    grouped = dp.is_initialized()
    device = torch.device("cuda", local)

    from image_denoising_amd import N2NTrainer, StructureTrainer, UNet

    ft = args.mode == "finetune"
    C = args.channels
    H = args.size or (512 if ft else 256)
    bs = args.bs or (16 if ft else 64)
    torch.manual_seed(0)
    iu = args.arch == "UNetImproved"
    if iu:
        from image_denoising_amd.improved_unet import ImprovedUNet

        net = ImprovedUNet(in_nc=C, out_nc=C, n_feature=48).to(device)
        net.set_precision(args.conv_precision)
    else:
        net = UNet(in_nc=C, out_nc=C, n_feature=48).to(device).set_precision(args.conv_precision)
    x6 = args.conv_precision == "fp32_x6"
    fwd_flops = iunet_fwd_flops if iu else unet_fwd_flops
    clean = synthetic_clean(bs * C, H, H, 1000 + rank, device).view(bs, C, H, H).contiguous()
    if ft:
        from image_denoising_amd.adapter import DenoiserWithAdapter
        from image_denoising_amd.finetune import FinetuneTrainer

        model = DenoiserWithAdapter(net, in_channels=C, hidden_channels=16).to(device)
        if args.precision == "bf16":
            if iu:
                raise SystemExit("--precision bf16 is built for the UNet base")
            model.base.set_inference_precision("bf16")
        tr = FinetuneTrainer(model, lr=1e-4, lambda_grad=0.1, distributed=grouped)
        g = torch.Generator(device="cpu").manual_seed(7 + rank)
        noisy = (clean + (25.0 / 255.0) * torch.randn(clean.shape, generator=g).to(device)).contiguous()
        step = lambda: tr.train_step(clean, noisy)
    elif args.mode == "n2n":
        tr = N2NTrainer(net, lr=3e-4, n_epoch=100, increase_ratio=2.0, seed=0, distributed=grouped)
        step = lambda: tr.train_step(clean, epoch=1)
    else:
        tr = StructureTrainer(net, lr=3e-4, n_epoch=100, distributed=grouped)
        g = torch.Generator(device="cpu").manual_seed(7 + rank)
        noisy = (clean + (25.0 / 255.0) * torch.randn(clean.shape, generator=g).to(device)).contiguous()
        step = lambda: tr.train_step(clean, noisy, epoch=1)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if grouped:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    loss_v = loss.cpu().tolist()
    # one profiled pair of steps after the timed region, on EVERY rank (the step all-reduces)
    recs, reps = step_profile(step)

    if args.breakdown and rank == 0 and args.mode == "n2n":
        breakdown(tr, clean, device)

    if rank == 0:
        ms_step = 1000.0 * elapsed / args.steps
        value = world * bs * args.steps / elapsed
        bf = ft and args.precision == "bf16"
        peak = PEAK_BF16_TFLOPS if bf else (PEAK_X6_TFLOPS if x6 else PEAK_FP32_TFLOPS)
        if args.mode == "n2n":  # fwd 256 + fwd/bwd 128
            ref_flops = bs * (fwd_flops(H, H, C) + 3 * fwd_flops(H // 2, H // 2, C))
        elif ft:  # frozen base forward + adapter fwd (864 flop/px) and bwd (~1728 flop/px, C=1)
            ref_flops = bs * (fwd_flops(H, H, C) + 3 * 864.0 * C * H * H)
        else:  # two fwd/bwd at full resolution
            ref_flops = bs * 2 * 3 * fwd_flops(H, H, C)
        shapes, weighted, ms3, by_op, executed = per_shape_roofline(recs, reps, peak)
        # the FLOPs the step's launches execute (the pair-pixel no-grad pass computes dec_conv1b
        # and the head at half the pixels): what step_tflops divides; ref_flops is SURVEY 8d's
        step_flops = executed if executed > 0 and not ft else ref_flops
        if shapes:  # the dominant in-step 3x3 launch shape (largest time per step)
            dom = shapes[0]
            kms, kflops = dom["avg_launch_ms"], dom["flops_per_launch"]
            kdesc = f"{dom['kernel']} {dom['op']} {dom['shape']} (in-step launch)"
            mode_tag = ("bf16" if bf else args.mode) + ("_iunet" if iu else "") + \
                (f"_c{C}" if C != 1 else "")
            traffic, traffic_src, traffic_by = pmc_step_traffic(dom, mode_tag)
        else:  # no 3x3 launch recorded: the isolated 96->96 shape
            timer = (time_dominant_kernel_bf16 if bf else
                     time_dominant_kernel_x6 if x6 else time_dominant_kernel)
            kms, kflops = timer(bs, H, H, device)
            kdesc = "96->96 3x3 @%dx%dx%d, isolated launch" % (bs, H, H)
            traffic, traffic_src, traffic_by = None, None, None
        achieved = kflops / (kms * 1e-3) / 1e12
        # the bound of the dominant launch: its arithmetic intensity (algorithmic FLOPs over the
        # fp32 activations it must move) against the machine balance peak / 8 TB/s -- the bf16
        # base's 3x3 convs (~217 FLOP/B against 312) are HBM-bound, the bf16x6 ones (52) are not
        alg_bytes = shapes[0]["algorithmic_bytes_per_launch"] if shapes else None
        hbm_bound = bool(alg_bytes) and kflops / alg_bytes < peak * 1e12 / (PEAK_HBM_GBS * 1e9)
        model = "ImprovedUNet(n_feature=48)" if iu else "UNet(n_feature=48)"
        if iu and not ft:
            workload = (f"{args.mode} step with arch_unet.ImprovedUNet(n_feature=48, depth=4, noise=True) "
                        f"(train.py:311-313), {bs}x{C}x{H}x{H} per GPU, Adam lr 3e-4")
        elif ft:
            workload = (f"BASELINE configs[4]: finetune.py adapter step, frozen {model} "
                        f"base (no_grad) + OutputAdapter(hidden 16), {bs}x{C}x{H}x{H} per GPU, "
                        f"L1 + 0.1*gradient_loss, Adam lr 1e-4, "
                        f"{'mixed-precision bf16 base' if args.precision == 'bf16' else 'fp32'}")
        elif args.mode == "structure":
            workload = (f"train.py Structure_loss step (train.py:355-368), UNet(n_feature=48), "
                        f"{bs}x{C}x{H}x{H} per GPU, Adam lr 3e-4")
        elif (C, bs) == (3, 32):
            workload = (f"BASELINE configs[3]: 3-channel N2N step, UNet(n_feature=48), "
                        f"{bs}x{C}x{H}x{H} per GPU, Adam lr 3e-4")
        else:
            workload = (f"BASELINE configs[1]: N2N step, UNet(n_feature=48), "
                        f"{bs}x{C}x{H}x{H} per GPU, Adam lr 3e-4")
        rec = {
            "metric": "training patches/sec (256x256x1, bs=64 per GPU, N2N loss + Adam)"
                      if args.mode == "n2n" and (C, bs, H) == (1, 64, 256) and not iu
                      else (f"finetune patches/sec ({H}x{H}x{C}, bs={bs} per GPU, frozen base + adapter)"
                            if ft else f"training patches/sec ({H}x{H}x{C}, bs={bs} per GPU, {args.mode}"
                                       f"{', ImprovedUNet' if iu else ''})"),
            "value": round(value, 2), "unit": "patches/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": ("bf16 (frozen base 3x3 convs; fp32 accumulate) + fp32 adapter" if bf else
                      "fp32 (3x3 convs: exact 3-piece bf16 split, 6 products, fp32 accumulate)"
                      if x6 else "fp32"),
            "data": "synthetic",
            "config": {"workload": workload,
                       "global_batch": bs * world, "patch": [H, H, C], "parallelism": f"dp{world}",
                       "collective": (f"{dist.get_backend()} all_reduce(sum) of the flat gradient per step"
                                      if grouped else "none (single process)")},
            "step_tflops": round(step_flops / (ms_step * 1e-3) / 1e12, 2),
            "step_frac_of_fp32_peak": round(step_flops / (ms_step * 1e-3) / 1e12 / PEAK_FP32_TFLOPS, 4),
            "step_flops_executed": step_flops, "step_flops_reference": ref_flops,
            "roofline": {"bound": "hbm" if hbm_bound else "mfma",
                         "kernel": kdesc + ("; bf16 MFMA" if bf else "; fp32 as 6 split-bf16 "
                                            "products, peak = bf16 dense / 6" if x6 else "; fp32 MFMA"),
                         **({"achieved": round(alg_bytes / (kms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                             "unit": "GB/s", "frac": round(alg_bytes / (kms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                             "mfma_achieved_tflops": round(achieved, 2), "mfma_peak_tflops": peak,
                             "mfma_frac": round(achieved / peak, 4)} if hbm_bound else
                            {"achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                             "frac": round(achieved / peak, 4)}),
                         "traffic": traffic,
                         "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                         "traffic_of": traffic_by,
                         "algorithmic_bytes_per_launch": shapes[0]["algorithmic_bytes_per_launch"]
                         if shapes else None,
                         "avg_launch_ms": round(kms, 4), "flops_per_launch": kflops,
                         "weighted_frac": round(weighted, 4) if weighted else None,
                         "weighted_over": "every 3x3 launch of the step (fwd, pair-pixel fwd, "
                                          "data and weight gradients), time-weighted",
                         "ms_3x3_per_step": round(ms3, 3),
                         "per_shape": [{k: v for k, v in d.items()
                                        if k != "algorithmic_bytes_per_launch" and not k.startswith("_")}
                                       for d in shapes],
                         "method": "one profiled step pair after the timed region, every launch "
                                   "bracketed by HIP events on its stream, single-stream "
                                   "(dn_profile_ops)"},
            "step_breakdown_ms": by_op,
            "loss": loss_v,
        }
        if args.mode == "n2n" and C == 1 and not iu and not args.no_eval:
            # "eval PSNR vs ref" (BASELINE metric): the trained weights denoise one 512x512 image
            # on the HIP path; the CPU leg runs the reference restatement on the same weights
            clean8, noisy8 = eval_image()
            ps, ss = hip_eval(net, clean8, noisy8)
            rec["eval"] = {"psnr": round(ps, 4), "ssim": round(ss, 5),
                           "image": "512x512 synthetic, gauss25, after the timed steps",
                           "noisy_psnr": round(float(10 * __import__("math").log10(
                               255.0 ** 2 / float(((noisy8.astype("f8") - clean8) ** 2).mean()))), 4)}
        if not args.no_cpu_baseline and not args.no_eval and world == 1 and args.mode == "n2n" and C == 1 and not iu:
            rec["cpu_baseline"] = cpu_baseline()
            ref_ps = oracle_eval_psnr(net.flat_params, clean8, noisy8)
            rec["cpu_baseline"]["eval_psnr"] = round(ref_ps, 4)
            rec["eval"]["psnr_ref_cpu"] = round(ref_ps, 4)
            rec["eval"]["psnr_abs_diff"] = round(abs(ps - ref_ps), 6)
        print(json.dumps(rec), flush=True)
    if grouped:
        dist.destroy_process_group()


def breakdown(tr, clean, device):
    """per-phase HIP-event timing of one step (stderr)"""
    from image_denoising_amd import _lib
    from image_denoising_amd.n2n import n2n_loss, n2n_subsample

    s = torch.cuda.current_stream(device)
    N, C, H, W = clean.shape
    b = tr._buffers(N, C, H, W, device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
    ev[0].record(s)
    _lib.call("dn_add_gauss_noise", _lib.ptr(clean), N, C * H * W, 0.098, None, 0, 0, 0,
              _lib.ptr(b["noisy"]), s.cuda_stream)
    sub1, sub2, rd = n2n_subsample(b["noisy"], None, seed=1, offset=1)
    ev[1].record(s)
    tr.net._run_forward(b["noisy"], b["den"], b["ws_den"])
    ev[2].record(s)
    tr.net._run_forward(sub1, b["out"], b["ws_grad"])
    ev[3].record(s)
    loss3, dout = n2n_loss(b["out"], sub2, b["den"], rd, 0.02)
    ev[4].record(s)
    tr.net._run_backward(dout, tr.grad, b["ws_grad"], N, H // 2, W // 2)
    ev[5].record(s)
    ev[6].record(s)
    ev[6].synchronize()
    names = ["noise+subsample", "fwd 256 (no grad)", "fwd 128 (saved)", "loss", "bwd 128"]
    for i, n in enumerate(names):
        print(f"  {n:22s} {ev[i].elapsed_time(ev[i + 1]):8.3f} ms", file=sys.stderr)


if __name__ == "__main__":
    main()
