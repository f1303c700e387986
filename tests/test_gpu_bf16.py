"""Mixed-precision (bf16 matrix cores) inference forward of the UNet — the frozen base of the
adapter finetune (BASELINE configs[4]) — vs the oracle emulating the same rounding.  GPU only."""
import numpy as np
import pytest
import torch

from oracle import adapter_ref, unet_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
# vs the bf16-emulating oracle (bf16-rounded operands of the 3x3 layers, fp64 accumulation):
# only the accumulation order differs, plus the odd activation whose fp32 value sits within an
# fp32 ulp of a bf16 rounding boundary and rounds the other way (2^-8 relative on that element,
# which reaches the output attenuated but, with ~1e6 activations per layer, not rarely)
EMU_TOL = 1e-2
# ... and element by element: a flip moves few outputs, so all but a small fraction of the
# elements must agree to 1e-3 of max |y| (an indexing error confined to a region would not)
EMU_ELEM_TOL, EMU_ELEM_FRAC = 1e-3, 2e-3
# vs the fp32 reference: the bf16 rounding itself (8-bit mantissa) through ~20 layers
FP32_TOL = 5e-2


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def assert_emulation_match(y, emu):
    """max error within EMU_TOL and at most EMU_ELEM_FRAC of the elements beyond EMU_ELEM_TOL
    (both relative to max |emu|)"""
    y = np.asarray(y, dtype=np.float64)
    emu = np.asarray(emu, dtype=np.float64)
    scale = max(np.abs(emu).max(), 1e-30)
    d = np.abs(y - emu) / scale
    frac = float((d > EMU_ELEM_TOL).mean())
    assert d.max() < EMU_TOL, d.max()
    assert frac <= EMU_ELEM_FRAC, (frac, d.max())


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("C,shape", [(1, (2, 64, 64)), (3, (1, 64, 96)), (1, (4, 256, 256))])
def test_unet_bf16_forward_vs_emulation(C, shape):
    from image_denoising_amd import UNet

    N, H, W = shape
    torch.manual_seed(0)
    net = UNet(C, C, 48).to(DEV).set_inference_precision("bf16")
    x = torch.rand(N, C, H, W, generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        y = net(x.to(DEV)).cpu()
        y2 = net(x.to(DEV)).cpu()
    assert torch.equal(y, y2)  # deterministic
    flat = net.flat_params.cpu().double()
    with torch.no_grad():
        emu = unet_ref.forward(flat, x.double(), C, C, bf16_3x3=True)
        ref = unet_ref.forward(flat, x.double(), C, C)
    assert_emulation_match(y.numpy(), emu.numpy())
    assert rel_err(y.numpy(), ref.numpy()) < FP32_TOL
    # and the fp32 path stays the fp32 path
    net.set_inference_precision("fp32")
    with torch.no_grad():
        y32 = net(x.to(DEV)).cpu()
    assert rel_err(y32.numpy(), ref.numpy()) < 1e-4


def test_finetune_step_with_bf16_base():
    from image_denoising_amd import DenoiserWithAdapter, FinetuneTrainer, UNet

    torch.manual_seed(0)
    base = UNet(1, 1, 48)
    torch.manual_seed(1)
    model = DenoiserWithAdapter(base, 1, 16).to(DEV)
    model.base.set_inference_precision("bf16")
    gen = torch.Generator().manual_seed(3)
    clean = torch.rand(2, 1, 64, 64, generator=gen)
    noisy = clean + 0.1 * torch.randn(2, 1, 64, 64, generator=gen)
    a0 = model.adapter.flat_params.cpu().clone()
    tr = FinetuneTrainer(model, lr=1e-4, lambda_grad=0.1)
    loss3 = tr.train_step(clean.to(DEV), noisy.to(DEV)).cpu().numpy()
    # oracle: the same step with the bf16-emulated base
    with torch.no_grad():
        base_out = unet_ref.forward(base.flat_params.cpu().double(), noisy.double(), 1, 1,
                                    bf16_3x3=True).float()
    p = a0.clone().requires_grad_(True)
    pred = adapter_ref.adapter_forward(p, noisy, base_out)
    l1, lg, loss = adapter_ref.finetune_loss(pred, clean, 0.1)
    loss.backward()
    assert rel_err(loss3, [l1.item(), lg.item(), loss.item()]) < EMU_TOL
    assert rel_err(tr.grad.cpu().numpy(), p.grad.numpy()) < 1e-2


def test_config4_full_size_finetune_step_properties():
    """BASELINE configs[4] at full size: 16 x 1 x 512^2 patches, frozen UNet base on the bf16
    matrix cores + OutputAdapter, one finetune.py:269-289 step.  Images are independent, so
    image 0's base output and adapted prediction are checked against the bf16-emulating oracle
    at full resolution; the adapter gradient must be finite and the weights must move."""
    from image_denoising_amd import DenoiserWithAdapter, FinetuneTrainer, UNet

    torch.manual_seed(0)
    base = UNet(1, 1, 48)
    torch.manual_seed(1)
    model = DenoiserWithAdapter(base, 1, 16).to(DEV)
    model.base.set_inference_precision("bf16")
    gen = torch.Generator().manual_seed(4)
    clean = torch.nn.functional.interpolate(torch.rand(16, 1, 64, 64, generator=gen), size=(512, 512),
                                            mode="bilinear", align_corners=False)
    noisy = clean + (25.0 / 255.0) * torch.randn(16, 1, 512, 512, generator=gen)
    a0 = model.adapter.flat_params.detach().cpu().clone()
    tr = FinetuneTrainer(model, lr=1e-4, lambda_grad=0.1)
    loss3 = tr.train_step(clean.to(DEV), noisy.to(DEV))
    torch.cuda.synchronize()
    l = loss3.cpu().numpy()
    assert np.isfinite(l).all() and l[2] > 0
    assert bool(torch.isfinite(tr.grad).all())
    assert not torch.equal(model.adapter.flat_params.detach().cpu(), a0)
    b = tr._bufs[next(iter(tr._bufs))]
    with torch.no_grad():
        emu = unet_ref.forward(base.flat_params.cpu().double(), noisy[:1].double(), 1, 1,
                               bf16_3x3=True).float()
    assert_emulation_match(b["base"][:1].cpu().numpy(), emu.numpy())
    pred = adapter_ref.adapter_forward(a0, noisy[:1], emu)
    assert_emulation_match(b["pred"][:1].cpu().numpy(), pred.detach().numpy())


def _conv_bf16(x, w, b, act, x_stride=None):
    """dn_conv2d_forward_bf16 on an NCHW fp32 input (optionally a channel view of a wider
    NHWC buffer: x_stride > Cin)."""
    from image_denoising_amd import _lib

    N, cin, H, W = x.shape
    cout = w.shape[0]
    xs = x_stride or cin
    buf = torch.zeros(N, H, W, xs)
    buf[..., :cin] = x.permute(0, 2, 3, 1)
    xg, wg, bg = buf.to(DEV), w.to(DEV), b.to(DEV)
    y = torch.empty(N, H, W, cout, device=DEV)
    pk = _lib.scratch(_lib.lib().dn_conv2d_bf16_pack_size(cin, cout), DEV)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("dn_conv2d_forward_bf16", xg.data_ptr(), xs, N, H, W, cin, wg.data_ptr(),
              bg.data_ptr(), cout, act, y.data_ptr(), cout, pk.data_ptr(), pk.numel(), s)
    return y.cpu().permute(0, 3, 1, 2)


# >= 1024 16x16 tiles with float4-aligned views and K % 4 == 0: the pipelined kernel
# (k_fwd_bf16p); the odd stride / K and the small grid: k_fwd_bf16
@pytest.mark.parametrize("cin,cout,N,H,W,xs", [
    (96, 96, 16, 128, 128, None), (48, 48, 16, 128, 128, None), (144, 96, 4, 256, 256, None),
    (96, 48, 16, 128, 120, 100), (36, 96, 16, 128, 128, None), (97, 96, 16, 128, 128, None),
    (96, 96, 2, 40, 40, None)])
def test_conv_bf16_vs_fp64_of_rounded_operands(cin, cout, N, H, W, xs):
    """bf16 products are exact in fp32, so against an fp64 conv of the bf16-rounded operands the
    only error is the fp32 accumulation order."""
    g = torch.Generator().manual_seed(cin * 7 + N)
    x = torch.randn(N, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
    b = torch.randn(cout, generator=g) * 0.1
    y = _conv_bf16(x, w, b, 1, xs)
    y2 = _conv_bf16(x, w, b, 1, xs)
    assert torch.equal(y, y2)
    xr, wr = x.bfloat16().double(), w.bfloat16().double()
    ref = torch.nn.functional.leaky_relu(
        torch.nn.functional.conv2d(xr, wr, b.double(), padding=1), 0.2)
    assert rel_err(y.numpy(), ref.numpy()) < 1e-5


def test_conv_bf16_48_rows8_tile():
    """48 -> 48 at 8 x 512^2 (>= 4096 tiles of 32 rows): the 8-rows-per-wave pipelined tile.
    Image 0 against an fp32 conv of the bf16-rounded operands (products exact, only the
    accumulation order differs)."""
    g = torch.Generator().manual_seed(48)
    x = torch.randn(8, 48, 512, 512, generator=g)
    w = torch.randn(48, 48, 3, 3, generator=g) * 0.05
    b = torch.randn(48, generator=g) * 0.1
    y = _conv_bf16(x, w, b, 1)
    xr, wr = x[:1].bfloat16().float(), w.bfloat16().float()
    ref = torch.nn.functional.leaky_relu(torch.nn.functional.conv2d(xr, wr, b, padding=1), 0.2)
    assert rel_err(y[:1].numpy(), ref.numpy()) < 1e-5
