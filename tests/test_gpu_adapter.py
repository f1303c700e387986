"""Adapter finetune path (adapter.py, finetune.py) on the HIP kernels vs the reference fixtures
and the CPU oracle, through the C-ABI.  Needs an MI355X."""
import numpy as np
import pytest
import torch

from oracle import adapter_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP32_TOL = 1e-4  # north_star: 1e-4 relative fp32


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _adapter(C, flat):
    from image_denoising_amd.adapter import OutputAdapter

    ad = OutputAdapter(in_channels=C, hidden_channels=16)
    ad.flat_params.copy_(torch.as_tensor(flat))
    return ad.to(DEV)


@pytest.mark.parametrize("C", [1, 3])
def test_adapter_fwd_bwd_vs_reference_fixture(golden, C):
    from image_denoising_amd.finetune import finetune_loss

    g = golden("adapter.npz")
    k = f"c{C}_"
    ad = _adapter(C, g[k + "params"])
    noisy, base, clean = (torch.from_numpy(g[k + n]).to(DEV) for n in ("noisy", "base", "clean"))
    out = torch.empty_like(base)
    ad._run_forward(noisy, base, out)
    assert rel_err(out.cpu().numpy(), g[k + "out"]) < FP32_TOL
    loss3, dpred = finetune_loss(out, clean, 0.1)
    assert rel_err(loss3.cpu().numpy(), g[k + "loss"]) < FP32_TOL
    grad = torch.empty_like(ad.flat_params)
    ad._run_backward(noisy, base, dpred, grad)
    assert rel_err(grad.cpu().numpy(), g[k + "grad"]) < FP32_TOL


@pytest.mark.parametrize("shape", [(2, 3, 37, 29), (1, 1, 5, 70), (3, 1, 64, 48)])
def test_adapter_ragged_shapes_vs_oracle(shape):
    N, C, H, W = shape
    gen = torch.Generator().manual_seed(sum(shape))
    torch.manual_seed(3)
    from image_denoising_amd.adapter import adapter_reference_init

    flat = adapter_reference_init(C) * 3.0  # larger weights: more ReLUs switch inside the tile
    noisy, base, dout = (torch.randn(N, C, H, W, generator=gen) for _ in range(3))
    p = flat.clone().requires_grad_(True)
    ref = adapter_ref.adapter_forward(p, noisy, base)
    ref.backward(dout)
    ad = _adapter(C, flat)
    out = torch.empty(N, C, H, W, device=DEV)
    ad._run_forward(noisy.to(DEV), base.to(DEV), out)
    assert rel_err(out.cpu().numpy(), ref.detach().numpy()) < FP32_TOL
    grad = torch.empty_like(ad.flat_params)
    ad._run_backward(noisy.to(DEV), base.to(DEV), dout.to(DEV), grad)
    assert rel_err(grad.cpu().numpy(), p.grad.numpy()) < FP32_TOL
    # deterministic: a second backward is bit-identical
    grad2 = torch.empty_like(grad)
    ad._run_backward(noisy.to(DEV), base.to(DEV), dout.to(DEV), grad2)
    assert torch.equal(grad, grad2)


@pytest.mark.parametrize("shape", [(3, 1, 17, 23), (2, 3, 2, 2), (4, 1, 128, 96)])
def test_finetune_loss_vs_oracle(shape):
    from image_denoising_amd.finetune import finetune_loss

    gen = torch.Generator().manual_seed(11)
    pred = torch.rand(shape, generator=gen)
    tgt = torch.rand(shape, generator=gen)
    tgt[..., ::3] = pred[..., ::3]  # exact ties: sgn(0) = 0 like torch
    p = pred.clone().requires_grad_(True)
    l1, lg, loss = adapter_ref.finetune_loss(p, tgt, 0.1)
    loss.backward()
    loss3, dpred = finetune_loss(pred.to(DEV), tgt.to(DEV), 0.1)
    assert rel_err(loss3.cpu().numpy(), [l1.item(), lg.item(), loss.item()]) < 1e-6
    assert rel_err(dpred.cpu().numpy(), p.grad.numpy()) < 1e-6


def test_finetune_step_vs_reference_fixture(golden):
    from image_denoising_amd.adapter import DenoiserWithAdapter
    from image_denoising_amd.arch_unet import UNet
    from image_denoising_amd.finetune import FinetuneTrainer

    g = golden("adapter.npz")
    torch.manual_seed(0)
    base = UNet(in_nc=1, out_nc=1, n_feature=48)
    torch.manual_seed(1)
    model = DenoiserWithAdapter(base, in_channels=1, hidden_channels=16).to(DEV)
    tr = FinetuneTrainer(model, lr=1e-4, lambda_grad=0.1)
    clean = torch.from_numpy(g["step_clean"]).to(DEV)
    noisy = torch.from_numpy(g["step_noisy"]).to(DEV)
    with torch.no_grad():
        pred = model(noisy)
    assert rel_err(pred.cpu().numpy(), g["step_pred"]) < FP32_TOL
    loss3 = tr.train_step(clean, noisy).cpu().numpy()
    assert rel_err(loss3, g["step_loss"]) < FP32_TOL
    assert rel_err(tr.grad.cpu().numpy(), g["step_grad"]) < FP32_TOL
    assert np.abs(model.adapter.flat_params.cpu().numpy() - g["step_post"]).max() < 1e-6


def test_autograd_path_matches_fused_step():
    """DenoiserWithAdapter + FinetuneLoss through torch autograd == the fused trainer's grad"""
    from image_denoising_amd.adapter import DenoiserWithAdapter
    from image_denoising_amd.arch_unet import UNet
    from image_denoising_amd.finetune import FinetuneLoss, FinetuneTrainer

    torch.manual_seed(5)
    model = DenoiserWithAdapter(UNet(1, 1, 48), 1, 16).to(DEV)
    gen = torch.Generator().manual_seed(6)
    clean = torch.rand(2, 1, 64, 96, generator=gen).to(DEV)
    noisy = (clean.cpu() + 0.1 * torch.randn(2, 1, 64, 96, generator=gen)).to(DEV)
    loss = FinetuneLoss(0.1)(model(noisy), clean)
    loss.backward()
    g_auto = torch.cat([p.grad.reshape(-1) for p in model.adapter.parameters()])
    tr = FinetuneTrainer(model, lr=1e-4, lambda_grad=0.1)
    l3 = tr.train_step(clean, noisy)
    assert abs(float(l3[2]) - float(loss)) <= 1e-6 * abs(float(loss))
    assert torch.equal(g_auto, tr.grad)
