"""One rank of the two-rank data-parallel check of tests/test_gpu_dist.py (not a test module).

Started as a fresh process per rank (RANK / WORLD_SIZE / MASTER_* in the environment) before
it touches the GPU; both ranks share the box's one GPU and talk over gloo.  Each rank runs the
PRODUCT N2NTrainer(distributed=True) -- broadcast at init, one all-reduce of the flat gradient
per step, 1/world folded into the fused Adam kernel -- for two steps on its contiguous shard of
a fixed global batch, then rank 0 writes what the test compares.

    python tests/dp_worker.py OUT.npz PRECISION            (two ranks, gloo)
    python tests/dp_worker.py OUT.npz PRECISION nccl       (one rank, RCCL)
    python tests/dp_worker.py OUT.npz PRECISION local      (no group; env-selected streams)
    python tests/dp_worker.py OUT.npz PRECISION grad       (one UNet forward + backward)
    python tests/dp_worker.py OUT.npz PRECISION igrad      (one ImprovedUNet forward + backward)

The `nccl` form is a ONE-rank RCCL group on the box's one GPU (RCCL does not put two ranks on
one device): the product trainer's broadcast and per-step all-reduce run through RCCL for real,
and the rank then repeats the two steps with distributed=False, so the test can require the two
runs to agree bit for bit (a one-rank all-reduce is the identity, the scale 1/world = 1).
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

B, H, W, STEPS = 4, 64, 64, 2
if os.environ.get("DPW_SHAPE"):  # "B,H,W": sizes on the large-grid kernels (k_c3w6, pipelined)
    B, H, W = (int(v) for v in os.environ["DPW_SHAPE"].split(","))


def global_inputs():
    """the global batch both the ranks and the single-process run use"""
    g = torch.Generator().manual_seed(4)
    clean = torch.rand(B, 1, H, W, generator=g)
    noisy = (clean + (25.0 / 255.0) * torch.randn(B, 1, H, W, generator=g)).contiguous()
    rd = torch.randint(0, 8, (B * (H // 2) * (W // 2),), generator=g, dtype=torch.uint8)
    return clean, noisy, rd


def build(prec, rank):
    from image_denoising_amd import UNet

    torch.manual_seed(0)
    net = UNet(in_nc=1, out_nc=1, n_feature=48).to("cuda").set_precision(prec)
    if rank == 1:  # replicas differ until the trainer's broadcast
        with torch.no_grad():
            net.flat_params.add_(0.5)
    return net


def run(tr, rank, world):
    clean, noisy, rd = global_inputs()
    b = B // world
    cells = (H // 2) * (W // 2)
    sl = slice(rank * b, (rank + 1) * b)
    losses = []
    for _ in range(STEPS):
        losses.append(tr.train_step(clean[sl].cuda(), epoch=1, noisy=noisy[sl].cuda(),
                                    rd_idx=rd[rank * b * cells:(rank + 1) * b * cells].cuda()))
    return torch.stack(losses)


def main_rccl(out, prec):
    from image_denoising_amd import N2NTrainer
    from image_denoising_amd import dist as dp

    world, rank, _ = dp.init_from_env("nccl", force=True)
    assert world == 1 and dp.is_initialized() and not dp.is_distributed()
    backend = dist.get_backend()
    net = build(prec, 0)
    tr = N2NTrainer(net, distributed=True)  # broadcast + all-reduce on the RCCL group
    assert tr.distributed
    losses = run(tr, 0, 1)
    grad, flat = tr.grad.cpu().numpy(), net.flat_params.detach().cpu().numpy()
    net2 = build(prec, 0)
    tr2 = N2NTrainer(net2, distributed=False)
    losses2 = run(tr2, 0, 1)
    torch.cuda.synchronize()
    np.savez(out, backend=np.array(backend), losses=losses.cpu().numpy(), grad=grad, flat=flat,
             losses_local=losses2.cpu().numpy(), grad_local=tr2.grad.cpu().numpy(),
             flat_local=net2.flat_params.detach().cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def main_local(out, prec):
    """one process, no group: the two steps under whatever DN_*_STREAMS the env sets"""
    from image_denoising_amd import N2NTrainer

    net = build(prec, 0)
    tr = N2NTrainer(net, distributed=False)
    losses = run(tr, 0, 1)
    torch.cuda.synchronize()
    np.savez(out, losses=losses.cpu().numpy(), grad=tr.grad.cpu().numpy(),
             flat=net.flat_params.detach().cpu().numpy())


def main_grad(out, prec):
    """one forward + backward of the product UNet (parameter and input gradients) under the
    env's plan overrides (DN_C1S_ALIGN)"""
    net = build(prec, 0)
    clean, noisy, _ = global_inputs()
    x = noisy.cuda().requires_grad_(True)
    y = net(x)
    (y ** 2).mean().backward()
    g = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    np.savez(out, y=y.detach().cpu().numpy(), g=g.cpu().numpy(), dx=x.grad.cpu().numpy())


def main_igrad(out, prec):
    """one forward + backward of the product ImprovedUNet (DPW_SHAPE B,H,W; C = 1) under the
    env's kernel routing (DN_W6_MIN_TILES, DN_X6_W6)"""
    from image_denoising_amd.improved_unet import ImprovedUNet

    torch.manual_seed(0)
    net = ImprovedUNet(in_nc=1, out_nc=1, n_feature=48).to("cuda").set_precision(prec)
    g = torch.Generator().manual_seed(5)
    x = torch.rand(B, 1, H, W, generator=g).cuda()
    y = net(x)
    (y ** 2).mean().backward()
    names = [n for n, _ in net.named_parameters()]
    grads = [p.grad.detach().reshape(-1).cpu().numpy() for _, p in net.named_parameters()]
    np.savez(out, y=y.detach().cpu().numpy(), names=np.array(names),
             **{f"g{i}": v for i, v in enumerate(grads)})


def main():
    out, prec = sys.argv[1], sys.argv[2]
    if len(sys.argv) > 3 and sys.argv[3] == "igrad":
        return main_igrad(out, prec)
    if len(sys.argv) > 3 and sys.argv[3] == "grad":
        return main_grad(out, prec)
    if len(sys.argv) > 3 and sys.argv[3] == "nccl":
        return main_rccl(out, prec)
    if len(sys.argv) > 3 and sys.argv[3] == "local":
        return main_local(out, prec)
    from image_denoising_amd import N2NTrainer
    from image_denoising_amd import dist as dp

    world, rank, _ = dp.init_from_env("gloo")
    assert world == 2 and dp.is_distributed()
    net = build(prec, rank)
    tr = N2NTrainer(net, distributed=True)
    losses = run(tr, rank, world)
    dp.allreduce_mean_(losses)  # global-batch loss = mean of the equal shards' means
    flat = net.flat_params.detach().cpu()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        np.savez(out, losses=losses.cpu().numpy(), grad=(tr.grad / world).cpu().numpy(),
                 flat0=gathered[0].numpy(), flat1=gathered[1].numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
