"""Evaluation path on the HIP kernels vs oracle/eval_ref.py (and the reference PSNR fixture).
Needs an MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from image_denoising_amd import _lib

    _lib.lib()


def test_psnr_matches_reference_fixture(golden):
    from image_denoising_amd.evaluation import calculate_psnr

    g = golden("eval_psnr.npz")
    for i in range(2):
        assert calculate_psnr(g["a"][i], g["b"][i]) == pytest.approx(float(g["psnr"][i]), rel=1e-6)


def test_psnr_identical_is_inf():
    from image_denoising_amd.evaluation import calculate_psnr

    a = np.full((16, 16), 7, np.uint8)
    assert calculate_psnr(a, a) == float("inf")


@pytest.mark.parametrize("shape", [(64, 48), (11, 11), (37, 53, 3), (40, 40, 1)])
def test_ssim_matches_oracle(shape):
    from image_denoising_amd.evaluation import calculate_ssim
    from oracle import eval_ref

    rng = np.random.default_rng(hash(shape) & 0xFFFF)
    a = rng.integers(0, 256, shape).astype(np.uint8)
    b = np.clip(a.astype(int) + rng.integers(-30, 31, shape), 0, 255).astype(np.uint8)
    assert calculate_ssim(a, b) == pytest.approx(eval_ref.calculate_ssim(a, b), rel=1e-10)
    assert calculate_ssim(a, a) == pytest.approx(1.0, abs=1e-12)


def test_l1_and_quantize_match_numpy():
    from image_denoising_amd import _lib

    g = torch.Generator().manual_seed(3)
    x = (torch.rand(3, 50, 70, generator=g) * 1.4 - 0.2)
    y = torch.rand(3, 50, 70, generator=g)
    xd, yd = x.to(DEV), y.to(DEV)
    parts = _lib.scratch(_lib.lib().dn_eval_partials_size(), DEV)
    out = torch.empty(1, dtype=torch.float64, device=DEV)
    _lib.call("dn_l1_mean", _lib.ptr(xd), _lib.ptr(yd), x.numel(), _lib.ptr(parts), _lib.ptr(out),
              _lib.stream_of(xd))
    assert float(out.item()) == pytest.approx(float((x.double() - y.double()).abs().mean()), rel=1e-12)
    q = torch.empty(x.shape, dtype=torch.uint8, device=DEV)
    from oracle import eval_ref

    for plus_half in (1, 0):
        _lib.call("dn_quantize_u8", _lib.ptr(xd), x.numel(), plus_half, _lib.ptr(q), _lib.stream_of(xd))
        want = eval_ref.quantize_full(x.numpy()) if plus_half else \
            np.clip(np.clip(x.numpy(), 0, 1) * np.float32(255.0), 0, 255).astype(np.uint8)
        assert np.array_equal(q.cpu().numpy(), want)


@pytest.mark.parametrize("hw", [(704, 704), (400, 530), (352, 352), (100, 90), (5, 7)])
def test_tile_extract_and_blend_bit_exact(hw):
    from image_denoising_amd import _lib
    from image_denoising_amd.evaluation import weight_mask
    from oracle import eval_ref

    h, w = hw
    ps, ov = (352, 64) if h > 7 else (16, 4)
    st = ps - ov
    rng = np.random.default_rng(h * 1000 + w)
    img = rng.integers(0, 256, (h, w)).astype(np.uint8)
    want_tiles = eval_ref.tile_extract(img, ps, ov)
    img_d = torch.from_numpy(img).to(DEV)
    tiles = torch.empty(want_tiles.shape, dtype=torch.float32, device=DEV)
    _lib.call("dn_tile_extract", _lib.ptr(img_d), 1, h, w, ps, st, _lib.ptr(tiles), _lib.stream_of(tiles))
    assert np.array_equal(tiles.cpu().numpy(), want_tiles)
    # blend of an arbitrary "prediction" (values outside [0,1] exercise the clamp)
    pred = (rng.random(want_tiles.shape, dtype=np.float32) * 1.3 - 0.15).astype(np.float32)
    den_w, p8_w = eval_ref.tile_blend(pred, h, w, ps, ov)
    pd = torch.from_numpy(pred).to(DEV)
    wm = torch.from_numpy(weight_mask(ps)).to(DEV)
    den = torch.empty((1, h, w), dtype=torch.float32, device=DEV)
    p8 = torch.empty((1, h, w), dtype=torch.uint8, device=DEV)
    _lib.call("dn_tile_blend", _lib.ptr(pd), 1, h, w, ps, st, _lib.ptr(wm), _lib.ptr(den),
              _lib.ptr(p8), _lib.stream_of(pd))
    assert np.array_equal(den.cpu().numpy()[0], den_w)
    assert np.array_equal(p8.cpu().numpy()[0], p8_w)


def _net():
    from image_denoising_amd import UNet

    torch.manual_seed(0)
    net = UNet(in_nc=1, out_nc=1, n_feature=48)
    with torch.no_grad():  # larger-than-init weights so the output is not ~constant
        for name, p in net.named_parameters():
            if name.endswith("weight"):
                p.mul_(8.0)
    return net.to(DEV).eval()


def test_denoise_full_matches_oracle():
    from image_denoising_amd.evaluation import calculate_psnr, calculate_ssim, denoise_full
    from oracle import eval_ref, unet_ref

    net = _net()
    rng = np.random.default_rng(7)
    noisy = rng.integers(0, 256, (96, 128)).astype(np.uint8)
    pred, p8, l1 = denoise_full(net, noisy)
    x = torch.from_numpy(noisy.astype(np.float32) / 255.0)[None, None]
    want = unet_ref.forward(net.flat_params.detach().cpu(), x, 1, 1)
    err = (pred.cpu() - want).abs().max() / want.abs().max()
    assert float(err) < 1e-4
    assert float(l1.item()) == pytest.approx(float((want - x).abs().mean()), rel=1e-4)
    w8 = eval_ref.quantize_full(want.numpy()[0])
    d = np.abs(p8.cpu().numpy().astype(int) - w8.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3  # rounding-boundary flips only
    clean = np.clip(noisy.astype(int) + rng.integers(-5, 6, noisy.shape), 0, 255).astype(np.uint8)
    assert calculate_psnr(p8[0], clean) == pytest.approx(eval_ref.psnr(p8.cpu().numpy()[0], clean), rel=1e-6)
    assert calculate_ssim(p8[0], clean) == pytest.approx(eval_ref.calculate_ssim(p8.cpu().numpy()[0], clean),
                                                         rel=1e-10)


def test_denoise_tiled_matches_oracle():
    from image_denoising_amd.evaluation import denoise_tiled
    from oracle import eval_ref, unet_ref

    net = _net()
    rng = np.random.default_rng(8)
    h, w = 400, 530
    noisy = rng.integers(0, 256, (h, w)).astype(np.uint8)
    den, p8, l1 = denoise_tiled(net, noisy, max_batch=4)
    tiles = torch.from_numpy(eval_ref.tile_extract(noisy, 352, 64))
    flat = net.flat_params.detach().cpu()
    pred = torch.cat([unet_ref.forward(flat, tiles[i:i + 1], 1, 1) for i in range(tiles.shape[0])])
    den_w, p8_w = eval_ref.tile_blend(pred.numpy(), h, w, 352, 64)
    assert np.abs(den.cpu().numpy()[0] - den_w).max() < 1e-4
    d = np.abs(p8.cpu().numpy()[0].astype(int) - p8_w.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3
    l1_w = np.mean([float((pred[i] - tiles[i]).abs().mean()) for i in range(tiles.shape[0])])
    assert float(l1.item()) == pytest.approx(l1_w, rel=1e-4)
