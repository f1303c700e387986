"""HIP path vs the CPU oracle / reference fixtures, through the C-ABI.  Needs an MI355X."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
FP32_TOL = 1e-4  # north_star: 1e-4 relative fp32 (denoised image, loss, per-kernel outputs)
# Parameter gradients of the whole network: per-layer max-abs error relative to that layer's
# max-abs gradient.  Layers far from the loss (enc_conv0: |g| ~ 1e-17 for L = mean(y^2)) are
# sums with heavy cancellation where any two fp32 summation orders (mkldnn vs MFMA tiles)
# differ by ~1e-4 relative; 5e-4 bounds that while still catching any indexing error (O(1)).
GRAD_TOL = 5e-4


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from image_denoising_amd import _lib

    _lib.lib()
    torch.manual_seed(1234)


def L():
    from image_denoising_amd import _lib

    return _lib


def test_gpu_library_built_from_these_sources():
    """the .so the GPU box loads is the one compiled from this tree's sources"""
    from image_denoising_amd import _build

    v = L().lib().dn_version().decode()
    assert v.endswith("src=" + _build.source_hash()), (v, _build.source_hash())


def S():
    return torch.cuda.current_stream().cuda_stream


def nhwc(t):  # NCHW -> NHWC contiguous
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


# ---------------------------------------------------------------------------------------
# neighbour sub-sampler (bit-exact)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["a", "b", "c"])
def test_subsample_matches_reference_fixture(golden, case):
    from image_denoising_amd import n2n

    g = golden("subsampler.npz")
    img = torch.from_numpy(g[f"{case}_img"]).to(DEV)
    rd = torch.from_numpy(g[f"{case}_rd"]).to(DEV)
    s1, s2, rd_used = n2n.n2n_subsample(img, rd)
    assert np.array_equal(s1.cpu().numpy(), g[f"{case}_sub1"])
    assert np.array_equal(s2.cpu().numpy(), g[f"{case}_sub2"])
    m1, m2 = n2n.rd_to_masks(rd)
    from oracle import n2n_ref

    o1, o2 = n2n_ref.masks_from_rd(g[f"{case}_rd"])
    assert np.array_equal(m1.cpu().numpy(), o1) and np.array_equal(m2.cpu().numpy(), o2)
    if case == "a":
        assert np.array_equal(m1.cpu().numpy(), g["a_mask1"])
    # drop-in generate_subimages(img, mask)
    assert torch.equal(n2n.generate_subimages(img, m1), s1)
    assert torch.equal(n2n.generate_subimages(img, m2), s2)


def test_subsample_philox_stream_bitexact():
    from image_denoising_amd import n2n
    from oracle import n2n_ref, philox

    img = torch.rand(3, 2, 64, 96, device=DEV)
    cells = 3 * 32 * 48
    s1, s2, rd = n2n.n2n_subsample(img, None, seed=11, offset=5, cell_base=777)
    ref_rd = philox.rd_idx(11, 5, cells, cell_base=777)
    assert np.array_equal(rd.cpu().numpy(), ref_rd)
    c1, c2 = n2n_ref.subimages_closed_form(img.cpu().numpy(), ref_rd)
    assert np.array_equal(s1.cpu().numpy(), c1) and np.array_equal(s2.cpu().numpy(), c2)
    # mask pair never coincides, one True per cell
    m1, m2 = n2n.rd_to_masks(rd)
    m1, m2 = m1.view(-1, 4), m2.view(-1, 4)
    assert (m1.sum(1) == 1).all() and (m2.sum(1) == 1).all() and not (m1 & m2).any()


def test_subsample_empty_batch():
    from image_denoising_amd import n2n

    img = torch.empty(0, 1, 8, 8, device=DEV)
    s1, s2, rd = n2n.n2n_subsample(img)
    assert s1.shape == (0, 1, 4, 4) and rd.numel() == 0


def test_gauss_noise_matches_philox_oracle():
    from image_denoising_amd.n2n import AugmentNoise
    from oracle import philox

    clean = torch.rand(2, 1, 32, 48, device=DEV)
    aug = AugmentNoise("gauss25", seed=9)
    noisy = aug.add_train_noise(clean, offset=4)
    z = philox.normal(9, 4, np.arange(clean.numel(), dtype=np.uint64)).reshape(clean.shape)
    ref = clean.cpu().numpy().astype(np.float64) + (25.0 / 255.0) * z
    assert np.abs(noisy.cpu().numpy() - ref).max() < 2e-6


@pytest.mark.parametrize("per_image", [False, True])
def test_poisson_noise_matches_philox_oracle(per_image):
    """dn_add_poisson_noise (train.py:102-111) bit-exact against the oracle's sampler (same
    Philox draws, same fp64 inversion), with one lam or one per image; and AugmentNoise's
    poisson styles route to it."""
    from image_denoising_amd import _lib
    from image_denoising_amd.n2n import AugmentNoise
    from oracle import philox

    torch.manual_seed(1)
    clean = torch.rand(3, 1, 40, 24, device=DEV)
    lam_img = torch.tensor([5.0, 30.0, 50.0], device=DEV) if per_image else None
    out = torch.empty_like(clean)
    _lib.call("dn_add_poisson_noise", clean.data_ptr(), 3, clean[0].numel(), 30.0,
              lam_img.data_ptr() if per_image else None, 21, 3, 0, out.data_ptr(),
              torch.cuda.current_stream().cuda_stream)
    ref = philox.poisson_noise(clean.cpu().numpy(), lam_img.cpu().numpy() if per_image else 30.0,
                               seed=21, offset=3)
    assert np.array_equal(out.cpu().numpy(), ref)
    aug = AugmentNoise("poisson30", seed=21)
    assert torch.equal(aug.add_train_noise(clean, offset=3), out) if not per_image else True


# ---------------------------------------------------------------------------------------
# op-level convolution kernels vs torch fp32 on the CPU
# ---------------------------------------------------------------------------------------
def _conv_ref(x, w, b, k, act):
    y = F.conv2d(x, w, b, padding=k // 2)
    return F.leaky_relu(y, 0.2) if act else y


@pytest.mark.parametrize("cin,cout,k,H,W", [
    (1, 48, 3, 32, 32), (3, 48, 3, 32, 48), (48, 48, 3, 32, 32), (48, 48, 3, 8, 8),
    (48, 48, 3, 4, 4), (96, 96, 3, 16, 16), (144, 96, 3, 16, 32), (97, 96, 3, 32, 32),
    (99, 96, 3, 32, 32), (96, 96, 1, 32, 32), (96, 1, 1, 32, 32), (96, 3, 1, 16, 16),
])
def test_conv_forward(cin, cout, k, H, W):
    _lib = L()
    N = 2
    x = torch.randn(N, cin, H, W)
    w = torch.randn(cout, cin, k, k) * 0.1
    b = torch.randn(cout) * 0.1
    act = 1 if cout > 3 else 0
    xg, wg, bg = nhwc(x).to(DEV), w.to(DEV), b.to(DEV)
    y = torch.empty(N, H, W, cout, device=DEV)
    pk = _lib.scratch(_lib.lib().dn_conv2d_pack_size(cin, cout, k, 0), DEV)
    _lib.call("dn_conv2d_forward", xg.data_ptr(), cin, N, H, W, cin, wg.data_ptr(), bg.data_ptr(),
              cout, k, act, y.data_ptr(), cout, pk.data_ptr(), pk.numel(), S())
    ref = _conv_ref(x, w, b, k, act)
    assert rel_err(nchw(y.cpu()).numpy(), ref.numpy()) < FP32_TOL


@pytest.mark.parametrize("cin,cout,k,H", [
    (48, 48, 3, 32), (96, 96, 3, 16), (144, 96, 3, 16), (48, 96, 3, 8), (96, 96, 1, 32),
    (96, 1, 1, 16), (96, 3, 1, 16),
])
@pytest.mark.parametrize("mode", ["plain", "mask", "accum"])
def test_conv_backward_data(cin, cout, k, H, mode):
    _lib = L()
    N, W = 2, H
    x = torch.randn(N, cin, H, W, requires_grad=True)
    w = torch.randn(cout, cin, k, k) * 0.1
    dz = torch.randn(N, cout, H, W)
    F.conv2d(x, w, None, padding=k // 2).backward(dz)
    ref = x.grad
    mask = torch.randn(N, cin, H, W)
    base = torch.randn(N, cin, H, W)
    if mode == "mask":
        ref = torch.where(mask > 0, ref, ref * 0.2)
    if mode == "accum":
        ref = ref + base
    dx = nhwc(base).to(DEV) if mode == "accum" else torch.zeros(N, H, W, cin, device=DEV)
    mg, dzg, wg = nhwc(mask).to(DEV), nhwc(dz).to(DEV), w.to(DEV)  # keep device tensors alive
    pk = _lib.scratch(_lib.lib().dn_conv2d_pack_size(cin, cout, k, 1), DEV)
    _lib.call("dn_conv2d_backward_data", dzg.data_ptr(), N, H, W, cout, wg.data_ptr(), cin, k,
              mg.data_ptr() if mode == "mask" else None, cin, 1 if mode == "accum" else 0,
              dx.data_ptr(), cin, pk.data_ptr(), pk.numel(), S())
    assert rel_err(nchw(dx.cpu()).numpy(), ref.numpy()) < FP32_TOL


@pytest.mark.parametrize("cin,cout,k,N,H,W", [
    (48, 48, 3, 2, 32, 32), (96, 96, 3, 2, 16, 16), (144, 96, 3, 2, 16, 16),
    (97, 96, 3, 2, 32, 32), (1, 48, 3, 2, 32, 32), (3, 48, 3, 1, 32, 32), (48, 48, 3, 3, 8, 8),
    (48, 48, 3, 4, 4, 4), (96, 96, 1, 2, 32, 32), (96, 1, 1, 2, 32, 32), (96, 3, 1, 2, 16, 16),
    (96, 96, 3, 8, 64, 64),
])
def test_conv_backward_weight(cin, cout, k, N, H, W):
    _lib = L()
    x = torch.randn(N, cin, H, W)
    w = (torch.randn(cout, cin, k, k) * 0.1).requires_grad_(True)
    b = torch.zeros(cout, requires_grad=True)
    dz = torch.randn(N, cout, H, W)
    F.conv2d(x, w, b, padding=k // 2).backward(dz)
    nbytes = _lib.lib().dn_conv2d_wgrad_slab_size(N, H, W, cin, cout, k)
    slab = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    dwb = torch.full((cout * cin * k * k + cout,), float("nan"), device=DEV)
    dzg, xg = nhwc(dz).to(DEV), nhwc(x).to(DEV)  # keep device tensors alive during the call
    _lib.call("dn_conv2d_backward_weight", dzg.data_ptr(), xg.data_ptr(), cin, N, H, W, cin, cout,
              k, dwb.data_ptr(), slab.data_ptr(), S())
    out = dwb.cpu().numpy()
    nw = cout * cin * k * k
    assert rel_err(out[:nw], w.grad.numpy().reshape(-1)) < FP32_TOL
    assert rel_err(out[nw:], b.grad.numpy()) < FP32_TOL


@pytest.mark.parametrize("cin,cout,H", [(48, 48, 4), (96, 96, 8), (96, 96, 16)])
def test_deconv_forward_backward(cin, cout, H):
    _lib = L()
    N, W = 2, H
    x = torch.randn(N, cin, H, W)
    xr = x.clone().requires_grad_(True)
    w = (torch.randn(cin, cout, 2, 2) * 0.1).requires_grad_(True)
    b = (torch.randn(cout) * 0.1).requires_grad_(True)
    y = F.conv_transpose2d(xr, w, b, stride=2)
    dy = torch.randn_like(y)
    y.backward(dy)
    # forward into a strided concat buffer at channel offset 0 (skip after it)
    stride = cout + 8
    yg = torch.zeros(N, 2 * H, 2 * W, stride, device=DEV)
    xg = nhwc(x).to(DEV)
    wg, bg = w.detach().to(DEV), b.detach().to(DEV)
    pf = _lib.scratch(_lib.lib().dn_deconv2x2_pack_size(cin, cout, 0), DEV)
    pb = _lib.scratch(_lib.lib().dn_deconv2x2_pack_size(cin, cout, 1), DEV)
    _lib.call("dn_deconv2x2_forward", xg.data_ptr(), N, H, W, cin, wg.data_ptr(), bg.data_ptr(),
              cout, yg.data_ptr(), stride, 0, pf.data_ptr(), pf.numel(), S())
    assert rel_err(nchw(yg[..., :cout].cpu()).numpy(), y.detach().numpy()) < FP32_TOL
    assert float(yg[..., cout:].abs().max()) == 0.0
    # data gradient (with and without the LeakyReLU mask)
    dyg = torch.zeros(N, 2 * H, 2 * W, stride, device=DEV)
    dyg[..., :cout] = nhwc(dy).to(DEV)
    dx = torch.empty(N, H, W, cin, device=DEV)
    _lib.call("dn_deconv2x2_backward_data", dyg.data_ptr(), stride, N, H, W, cout, wg.data_ptr(),
              cin, None, dx.data_ptr(), pb.data_ptr(), pb.numel(), S())
    assert rel_err(nchw(dx.cpu()).numpy(), xr.grad.numpy()) < FP32_TOL
    mask = torch.randn(N, cin, H, W)
    mg = nhwc(mask).to(DEV)
    _lib.call("dn_deconv2x2_backward_data", dyg.data_ptr(), stride, N, H, W, cout, wg.data_ptr(),
              cin, mg.data_ptr(), dx.data_ptr(), pb.data_ptr(), pb.numel(), S())
    refm = torch.where(mask > 0, xr.grad, xr.grad * 0.2)
    assert rel_err(nchw(dx.cpu()).numpy(), refm.numpy()) < FP32_TOL
    # weight gradient
    nbytes = _lib.lib().dn_deconv2x2_wgrad_slab_size(N, H, W, cin, cout)
    slab = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    dwb = torch.empty(cin * cout * 4 + cout, device=DEV)
    _lib.call("dn_deconv2x2_backward_weight", dyg.data_ptr(), stride, xg.data_ptr(), N, H, W, cin,
              cout, dwb.data_ptr(), slab.data_ptr(), S())
    out = dwb.cpu().numpy()
    assert rel_err(out[:cin * cout * 4], w.grad.numpy().reshape(-1)) < FP32_TOL
    assert rel_err(out[cin * cout * 4:], b.grad.numpy()) < FP32_TOL


@pytest.mark.parametrize("ties", [False, True])
def test_maxpool_forward_backward(ties):
    _lib = L()
    N, C, H, W = 2, 48, 16, 24
    x = torch.randint(-2, 3, (N, C, H, W)).float() if ties else torch.randn(N, C, H, W)
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 2)
    dy = torch.randn_like(y)
    y.backward(dy)
    xg = nhwc(x).to(DEV)
    yg = torch.zeros(N, H // 2, W // 2, 2 * C, device=DEV)  # into the second half of a concat
    _lib.call("dn_maxpool2x2_forward", xg.data_ptr(), N, H, W, C, yg.data_ptr(), 2 * C, C, S())
    assert torch.equal(nchw(yg[..., C:].cpu()), y.detach())
    dyg = torch.zeros(N, H // 2, W // 2, 2 * C, device=DEV)
    dyg[..., C:] = nhwc(dy).to(DEV)
    for act in (0, 1):
        dx = torch.empty(N, H, W, C, device=DEV)
        _lib.call("dn_maxpool2x2_backward", xg.data_ptr(), N, H, W, C, dyg.data_ptr(), 2 * C, C,
                  act, dx.data_ptr(), S())
        ref = xr.grad if not act else torch.where(x > 0, xr.grad, xr.grad * 0.2)
        assert torch.equal(nchw(dx.cpu()), ref), f"act={act}"


# ---------------------------------------------------------------------------------------
# whole U-Net vs reference fixtures
# ---------------------------------------------------------------------------------------
def _net(C, prec="fp32"):
    from image_denoising_amd import UNet

    torch.manual_seed(0)
    return UNet(in_nc=C, out_nc=C, n_feature=48).to(DEV).set_precision(prec)


# the whole-network parity tests run both 3x3-conv arithmetics (DN_PREC_*): fp32 on the fp32
# matrix cores and the split-bf16 fp32 ("fp32_x6") on the bf16 ones, at the same tolerances
PRECS = ["fp32", "fp32_x6"]


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("C,name", [(1, "unet_c1.npz"), (3, "unet_c3.npz")])
def test_unet_forward_backward_vs_reference(golden, C, name, prec):
    """Output within 1e-4 of the reference; parameter gradients as close to the exact (fp64)
    gradient as the reference's own fp32 gradients are."""
    from oracle.unet_ref import forward, layer_table

    g = golden(name)
    net = _net(C, prec)
    x = torch.from_numpy(g["x"]).to(DEV)
    with torch.no_grad():
        y0 = net(x)
    assert rel_err(y0.cpu().numpy(), g["y"]) < FP32_TOL
    y = net(x)
    assert torch.equal(y.detach(), y0)  # grad path == no-grad path
    (y ** 2).mean().backward()
    grad = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).cpu().numpy()
    # exact gradient in fp64 on the CPU
    p64 = net.flat_params.detach().cpu().double().requires_grad_(True)
    y64 = forward(p64, torch.from_numpy(g["x"]).double(), C, C)
    (y64 ** 2).mean().backward()
    g64 = p64.grad.numpy()
    if "grad" in g:
        ref32, idx = g["grad"], np.arange(g64.size)
    else:
        idx = g["grad_idx"]
        ref32 = np.zeros_like(g64)
        ref32[idx] = g["grad_sample"]
    sel = np.zeros(g64.size, bool)
    sel[idx] = True
    off = 0
    for name_, ws, bl, _ in layer_table(C, C):
        n = int(np.prod(ws)) + bl
        m = sel[off:off + n]
        if m.any():
            t = g64[off:off + n][m]
            e_gpu = rel_err(grad[off:off + n][m], t)
            # LeakyReLU slope flips at pre-activations within rounding of 0 make per-layer
            # max-norm errors vs fp64 depend on the fp32 forward's rounding: the reference's
            # own fp32 grads move by ~1e-4 between mkldnn thread counts.  The rounding-only
            # check is test_unet_unit_gain_fwd_bwd_vs_fp64 (matched masks, < 2e-5).
            assert e_gpu < 1e-3, (name_, e_gpu)
        off += n
    norms = [float(p.grad.norm()) for p in net.parameters()]
    assert rel_err(norms, g["grad_norms"]) < FP32_TOL


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("C,name", [(1, "unet_c1.npz"), (3, "unet_c3.npz")])
def test_unet_input_grad_vs_reference(golden, C, name, prec):
    """dL/dx through the boundary (dn_unet_backward's dx) against the reference module's own
    autograd (fixture dx, arch_unet.py:194-260), with trainable and with frozen parameters."""
    g = golden(name)
    net = _net(C, prec)
    x = torch.from_numpy(g["x"]).to(DEV).requires_grad_(True)
    y = net(x)
    (y ** 2).mean().backward()
    assert x.grad is not None and x.grad.shape == x.shape
    assert rel_err(x.grad.cpu().numpy(), g["dx"]) < FP32_TOL
    assert all(p.grad is not None for p in net.parameters())
    # frozen parameters (the adapter-finetune base, finetune.py:255-262): only dx flows
    for p in net.parameters():
        p.requires_grad_(False)
    x2 = torch.from_numpy(g["x"]).to(DEV).requires_grad_(True)
    (net(x2) ** 2).mean().backward()
    assert torch.equal(x2.grad, x.grad)
    # and no input gradient requested: the inference path, no graph
    with torch.no_grad():
        assert not net(x2).requires_grad


def _pair_mask(rd, N, H, W):
    """bool [N,1,H,W]: the two pixels pair[rd][0], pair[rd][1] of every 2x2 cell"""
    from oracle import n2n_ref

    m1, m2 = n2n_ref.masks_from_rd(rd.numpy().astype(np.int64))
    cells = (m1 | m2).reshape(N, H // 2, W // 2, 2, 2)  # k = 2*dy + dx
    return cells.transpose(0, 1, 3, 2, 4).reshape(N, 1, H, W)


def _rd_set(kind, n, g):
    """per-cell pair choices: all eight (mixed), only horizontal pairs (rd 0/3/4/7: F(2,3) tiles
    along x in the Winograd pass) or only vertical ones (1/2/5/6: tiles along y)"""
    r = torch.randint(0, 8, (n,), generator=g, dtype=torch.uint8)
    if kind == "h":
        r = torch.tensor([0, 3, 4, 7], dtype=torch.uint8)[(r % 4).long()]
    elif kind == "v":
        r = torch.tensor([1, 2, 5, 6], dtype=torch.uint8)[(r % 4).long()]
    return r


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("rdk", ["mixed", "h", "v"])
@pytest.mark.parametrize("C,N,H,W", [(1, 2, 64, 64), (3, 1, 64, 96), (1, 8, 128, 128),
                                     (3, 4, 128, 160)])
def test_unet_forward_n2n_pair_pixels(C, N, H, W, prec, rdk):
    """dn_unet_forward_n2n (the N2N step's no-grad pass) = the full forward at the pair pixels;
    with fp32_x6 nothing else is written (dec_conv1b and the head run on the pair pixels only).
    From one round of 8 x 16 tiles (8 x 128^2 and up) the pair pass's dec_conv1b runs the
    Winograd kernel k_c3w6s (F(2,3) along x for horizontal pairs, along y for vertical ones)
    while the full forward runs k_c3w6 along x: the same fp32-accurate arithmetic class, so
    they agree to 2e-5 of max |y| (unit-gain weights: every level contributes); below that both
    run direct kernels with the same per-pixel arithmetic and agree bit for bit."""
    net = _net(C, prec)
    _unit_gain(net)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(N, C, H, W, generator=g).to(DEV)
    rd = _rd_set(rdk, N * (H // 2) * (W // 2), g).to(DEV)
    ws = net._workspace(N, H, W, with_backward=False, fresh=True)
    full = torch.empty(N, C, H, W, device=DEV)
    net._run_forward(x, full, ws)
    den = torch.full((N, C, H, W), float("nan"), device=DEV)
    net._run_forward_n2n(x, den, ws, rd)
    sel = torch.from_numpy(_pair_mask(rd.cpu(), N, H, W)).to(DEV).expand(N, C, H, W)
    assert bool(torch.isfinite(den[sel]).all())
    winograd = prec == "fp32_x6" and N * (H // 8) * (W // 16) >= 512
    if winograd:
        err = (den[sel] - full[sel]).abs().max().item()
        assert err <= 2e-5 * full.abs().max().item(), err
    else:
        assert torch.equal(den[sel], full[sel])
    if prec == "fp32_x6":
        assert bool(torch.isnan(den[~sel]).all())


@pytest.mark.parametrize("prec", ["fp32", "fp32_x6", "bf16"])
def test_unet_forward_prepacked_equals_forward(prec):
    """dn_unet_pack_weights once, then dn_unet_forward_prepacked on several batches: bit for bit
    the forward that packs per call (SURVEY §8b persistent packed weights), for each arithmetic;
    and the images really persist: after the parameters change, a prepacked forward still gives
    the old weights' result while a packing forward gives the new one."""
    net = _net(1, "fp32" if prec == "bf16" else prec)
    if prec == "bf16":
        net.set_inference_precision("bf16")
    g = torch.Generator().manual_seed(11)
    N, H, W = 2, 64, 96
    ws = net._workspace(N, H, W, with_backward=False, fresh=True)
    ws2 = net._workspace(N, H, W, with_backward=False, fresh=True).clone()
    xs = [torch.rand(N, 1, H, W, generator=g).to(DEV) for _ in range(2)]
    net._pack_weights(ws, N, H, W)
    for x in xs:
        ref, pre = torch.empty_like(x), torch.empty_like(x)
        net._run_forward_inference(x, ref, ws2)
        net._run_forward_prepacked(x, pre, ws)
        assert torch.equal(pre, ref)
    old = torch.empty_like(xs[0])
    net._run_forward_inference(xs[0], old, ws2)
    with torch.no_grad():
        net.flat_params.mul_(1.5)
    pre, new = torch.empty_like(old), torch.empty_like(old)
    net._run_forward_inference(xs[0], new, ws2)
    assert not torch.equal(new, old)
    net._run_forward_prepacked(xs[0], pre, ws)  # images of the old weights, new biases
    assert not torch.equal(pre, new)
    net._pack_weights(ws, N, H, W)
    net._run_forward_prepacked(xs[0], pre, ws)
    assert torch.equal(pre, new)


@pytest.mark.parametrize("unit_gain", [False, True])
@pytest.mark.parametrize("rdk", ["h", "v", "mixed"])
def test_unet_forward_n2n_pair_pixels_vs_oracle(rdk, unit_gain):
    """The Winograd pair pass (8 x 128^2: k_c3w6s for both tile orientations) against the CPU
    oracle of arch_unet.UNet.forward in fp64 at the pair pixels: 1e-4 of max |y| (north_star's
    fp32 tolerance on the denoised image).  At the reference initialisation the deep paths are
    ~1e-10 of y, so the unit-gain variant (every level O(1), _unit_gain) is the one that checks
    the encoder and the bottleneck through the pair pass too."""
    from oracle import unet_ref

    C, N, H, W = 1, 8, 128, 128
    net = _net(C, "fp32_x6")
    if unit_gain:
        _unit_gain(net)
    g = torch.Generator().manual_seed(5)
    x = torch.rand(N, C, H, W, generator=g)
    rd = _rd_set(rdk, N * (H // 2) * (W // 2), g)
    ws = net._workspace(N, H, W, with_backward=False, fresh=True)
    den = torch.full((N, C, H, W), float("nan"), device=DEV)
    net._run_forward_n2n(x.to(DEV), den, ws, rd.to(DEV))
    with torch.no_grad():
        ref = unet_ref.forward(net.flat_params.detach().cpu().double(), x.double(), C, C)
    sel = torch.from_numpy(_pair_mask(rd, N, H, W))
    d, r = den.cpu().double()[sel], ref[sel]
    assert (d - r).abs().max().item() <= 1e-4 * r.abs().max().item()


def _unit_gain(net, seed=0):
    """weights x10 (undoing the reference's x0.1 init) and random biases: every U-Net level
    then contributes O(1) to the output, so a fault in any level shows up in y and in every
    gradient.  With the reference init the deep paths are ~1e-10 of y."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if name.endswith("weight"):
                p.mul_(10.0)
            else:
                p.copy_((torch.randn(p.shape, generator=g) * 0.1).to(p.device))


ACT_NAMES = ["a0", "a1", "a2", "a3", "a4", "a5", "a6", "d2a", "d3a", "d4a", "d5a", "d2b", "d3b",
             "d4b", "d5b", "d1a", "d1b", "na", "nb"]
# dn_unet_debug_buffers order of the forward buffers
FWD_BUFS = ["c1", "a0", "a1", "c2", "c3", "c4", "c5", "a2", "a3", "a4", "a5", "p5", "a6",
            "d2a", "d3a", "d4a", "d5a", "d2b", "d3b", "d4b", "d5b", "d1a", "d1b", "na", "nb"]


def _ws_activations(net, ws, N, H, W):
    """the saved activations (ACT_NAMES, NCHW, CPU) of a with_backward workspace after a forward"""
    desc = (ctypes.c_int64 * 300)()
    n = ctypes.c_int()
    L().call("dn_unet_debug_buffers", ctypes.byref(net._cfg), N, H, W, 1, desc, 100,
             ctypes.byref(n))
    torch.cuda.synchronize()
    wsf = ws.view(torch.float32)
    acts = {}
    for i, name in enumerate(FWD_BUFS):
        off, st, lvl = desc[3 * i], desc[3 * i + 1], desc[3 * i + 2]
        h, w = H >> lvl, W >> lvl
        if name in ACT_NAMES:
            acts[name] = wsf[off:off + N * h * w * st].view(N, h, w, st).permute(0, 3, 1, 2).cpu().clone()
    return acts


def _device_activations(net, x, r):
    """run the HIP forward+backward on a debug-visible workspace; return (y, dflat, acts)"""
    _lib = L()
    N, C, H, W = x.shape
    desc = (ctypes.c_int64 * 300)()
    n = ctypes.c_int()
    _lib.call("dn_unet_debug_buffers", ctypes.byref(net._cfg), N, H, W, 1, desc, 100,
              ctypes.byref(n))
    ws = net._workspace(N, H, W, True, fresh=True)
    y = torch.empty(N, net.out_nc, H, W, device=DEV)
    net._run_forward(x.to(DEV).contiguous(), y, ws)
    dy = r.to(DEV).contiguous()
    dflat = torch.empty_like(net.flat_params)
    dx = torch.full((N, C, H, W), float("nan"), device=DEV)
    net._run_backward(dy, dflat, ws, N, H, W, dx=dx)
    torch.cuda.synchronize()
    _device_activations.dx = dx.cpu()
    wsf = ws.view(torch.float32)
    acts = {}
    for i, name in enumerate(FWD_BUFS):
        off, st, lvl = desc[3 * i], desc[3 * i + 1], desc[3 * i + 2]
        h, w = H >> lvl, W >> lvl
        if name in ACT_NAMES:
            acts[name] = wsf[off:off + N * h * w * st].view(N, h, w, st).permute(0, 3, 1, 2).cpu().clone()
    return y.cpu(), dflat.cpu(), acts


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("C,N,H,W", [(1, 2, 64, 64), (1, 1, 32, 32), (1, 3, 32, 96),
                                     (3, 2, 64, 32), (1, 2, 128, 128), (1, 4, 128, 128),
                                     (3, 4, 128, 128)])
def test_unet_unit_gain_fwd_bwd_vs_fp64(C, N, H, W, prec):
    """Every level contributes O(1) (unit-gain weights).  Forward vs fp64 within 1e-4; all 50
    parameter gradients vs an fp64 backward that takes LeakyReLU slopes and pool routing from
    the device's own fp32 activations (so only the rounding of the linear ops remains).
    (4 x 128^2: one full round of 8 x 16 tiles at the top level, so the Winograd kernels run
    there -- dec_conv1a's one-channel tail as one MFMA per fragment pair at C = 1, the packed
    four-channel tail at C = 3 -- as in the bench step.)"""
    from oracle.unet_ref import forward, layer_table

    net = _net(C, prec)
    _unit_gain(net)
    x = torch.rand(N, C, H, W, generator=torch.Generator().manual_seed(1))
    r = torch.randn(N, C, H, W, generator=torch.Generator().manual_seed(2))
    y, gg, acts = _device_activations(net, x, r)
    flat = net.flat_params.detach().cpu()
    dx = _device_activations.dx
    p64 = flat.double().requires_grad_(True)
    x64 = x.double().requires_grad_(True)
    y64 = forward(p64, x64, C, C, masks=acts)
    assert rel_err(y.numpy(), y64.detach().numpy()) < FP32_TOL
    (y64 * r.double()).sum().backward()
    g64 = p64.grad.numpy()
    assert rel_err(dx.numpy(), x64.grad.numpy()) < 2e-5
    gg = gg.numpy()
    off = 0
    for name_, ws, bl, _ in layer_table(C, C):
        n = int(np.prod(ws)) + bl
        e = rel_err(gg[off:off + n], g64[off:off + n])
        assert e < 2e-5, (name_, e)
        off += n


def test_unet_rejects_bad_shapes():
    net = _net(1)
    with pytest.raises(ValueError):
        net(torch.rand(1, 1, 48, 64, device=DEV))
    with pytest.raises(ValueError):
        net(torch.rand(1, 3, 64, 64, device=DEV))


# ---------------------------------------------------------------------------------------
# losses, Adam, the full N2N step
# ---------------------------------------------------------------------------------------
def test_n2n_loss_vs_oracle(golden):
    from image_denoising_amd import n2n
    from oracle import n2n_ref

    g = golden("n2n_step.npz")
    out = torch.from_numpy(g["out"]).to(DEV)
    noisy = torch.from_numpy(g["noisy"]).to(DEV)
    rd = torch.from_numpy(g["rd"]).to(DEV)
    _, sub2, _ = n2n.n2n_subsample(noisy, rd)
    den = torch.from_numpy(g["den"]).to(DEV)
    loss3, dout = n2n.n2n_loss(out, sub2, den, rd, float(g["lam"]))
    l = loss3.cpu().numpy()
    assert abs(l[0] - float(g["loss1"])) <= 1e-5 * float(g["loss1"])
    assert abs(l[1] - float(g["loss2"])) <= 1e-4 * float(g["loss2"]) + 1e-12
    assert abs(l[2] - float(g["loss"])) <= 1e-5 * float(g["loss"])
    assert rel_err(dout.cpu().numpy(), g["dout"]) < 1e-5
    # oracle restatement agrees too
    r = n2n_ref.n2n_loss(g["out"], sub2.cpu().numpy(), g["den"], g["rd"], float(g["lam"]))
    assert abs(r[2] - float(l[2])) <= 1e-5 * r[2]


def test_structure_loss_vs_reference(golden):
    from image_denoising_amd.util import Structure_loss

    g = golden("structure_loss.npz")
    pred = torch.from_numpy(g["pred"]).to(DEV).requires_grad_(True)
    pred2 = torch.from_numpy(g["pred2"]).to(DEV).requires_grad_(True)
    tgt = torch.from_numpy(g["target"]).to(DEV)
    L_ = Structure_loss()(pred, pred2, tgt)
    L_.backward()
    assert abs(float(L_) - float(g["loss"])) < 1e-6
    assert rel_err(pred.grad.cpu().numpy(), g["dpred"]) < 1e-5
    assert rel_err(pred2.grad.cpu().numpy(), g["dpred2"]) < 1e-5


def test_adam_matches_torch_adam():
    from image_denoising_amd.optim import FlatAdam

    n = 100_003
    p0 = torch.randn(n) * 0.05
    pt = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([pt], lr=3e-4)
    pg = p0.clone().to(DEV)
    fa = FlatAdam(pg, lr=3e-4)
    for _ in range(3):
        g = torch.randn(n) * torch.logspace(-9, 0, n)
        pt.grad = g.clone()
        opt.step()
        fa.step(g.to(DEV))
    assert torch.allclose(pg.cpu(), pt.detach(), rtol=0, atol=1e-7)
    # same formulas as ATen's vectorised CPU kernels; last-bit differences remain where the
    # CPU build contracts a*b+c differently
    assert float((pg.cpu() != pt.detach()).float().mean()) < 0.05


@pytest.mark.parametrize("prec", PRECS)
def test_n2n_step_vs_reference(golden, prec):
    from image_denoising_amd import N2NTrainer
    from image_denoising_amd.arch_unet import reference_init

    g = golden("n2n_step.npz")
    net = _net(1, prec)
    torch.manual_seed(0)
    pre = reference_init(1, 1, 48).numpy()
    tr = N2NTrainer(net, lr=3e-4, n_epoch=100, increase_ratio=2.0)
    noisy = torch.from_numpy(g["noisy"]).to(DEV)
    rd = torch.from_numpy(g["rd"]).to(DEV)
    loss3 = tr.train_step(noisy, epoch=1, rd_idx=rd, noisy=noisy).cpu().numpy()
    assert abs(loss3[0] - float(g["loss1"])) <= 1e-4 * float(g["loss1"])
    assert abs(loss3[2] - float(g["loss"])) <= 1e-4 * float(g["loss"])
    grad = tr.grad.cpu().numpy()
    assert rel_err(grad[g["grad_idx"]], g["grad_sample"]) < FP32_TOL
    post = net.flat_params.cpu().numpy()
    upd, ref_upd = post[g["post_idx"]] - pre[g["post_idx"]], g["post_sample"] - pre[g["post_idx"]]
    bad = np.abs(upd - ref_upd) > 1e-6
    assert bad.mean() < 2e-3, bad.mean()
    assert np.abs(upd - ref_upd).max() <= 6.1e-4  # never more than 2*lr apart


@pytest.mark.parametrize("prec", PRECS)
def test_n2n_step_deterministic(prec):
    from image_denoising_amd import N2NTrainer

    clean = torch.rand(4, 1, 64, 64, device=DEV)
    res = []
    for _ in range(2):
        net = _net(1, prec)
        tr = N2NTrainer(net, seed=3)
        for e in range(2):
            tr.train_step(clean, epoch=1)
        res.append((net.flat_params.clone(), tr.grad.clone()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_n2n_step_streams_equal_one_stream():
    """the bench step's concurrency (weight gradients and slab reductions on the library's side
    streams) against every library launch on the caller's stream (dn_profile_ops on), at a size
    where the streams overlap (16 x 256^2): the gradient and the updated weights bit-identical"""
    from image_denoising_amd import N2NTrainer, _lib

    clean = torch.rand(16, 1, 256, 256, generator=torch.Generator().manual_seed(5)).to(DEV)
    res = []
    try:
        for one_stream in (False, True):
            _lib.profile_ops(one_stream)
            net = _net(1, "fp32_x6")
            tr = N2NTrainer(net, seed=3)
            tr.train_step(clean, epoch=1)
            torch.cuda.synchronize()
            res.append((net.flat_params.detach().clone(), tr.grad.clone()))
    finally:
        _lib.profile_ops(False)
    assert torch.isfinite(res[0][1]).all()
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][0], res[1][0])


@pytest.mark.parametrize("style", ["gauss25", "poisson30", "poisson5_50", "gauss5_50"])
def test_n2n_step_noise_styles(style):
    """N2NTrainer(noise_style=...) synthesises the step's noisy batch with the chosen train.py
    --noisetype (gauss25 equal to the default noise_std path) and steps on it."""
    from image_denoising_amd import N2NTrainer
    from oracle import philox

    clean = torch.rand(4, 1, 64, 64, device=DEV)
    tr = N2NTrainer(_net(1, "fp32_x6"), seed=5, noise_style=style)
    loss3 = tr.train_step(clean, epoch=1)
    noisy = tr._bufs[next(iter(tr._bufs))]["noisy"].cpu()
    assert np.isfinite(loss3.cpu().numpy()).all()
    if style == "gauss25":
        tr0 = N2NTrainer(_net(1, "fp32_x6"), seed=5)
        tr0.train_step(clean, epoch=1)
        assert torch.equal(tr0._bufs[next(iter(tr0._bufs))]["noisy"].cpu(), noisy)
    elif style == "poisson30":
        ref = philox.poisson_noise(clean.cpu().numpy(), 30.0, seed=5, offset=0)
        assert np.array_equal(noisy.numpy(), ref)
    elif style == "poisson5_50":  # one lam per image of the global batch, seeded by the step
        g = torch.Generator(device="cpu").manual_seed(5 * 1000003 + 0)
        lam = (torch.rand(4, generator=g) * (50.0 - 5.0) + 5.0).numpy()
        ref = philox.poisson_noise(clean.cpu().numpy(), lam, seed=5, offset=0)
        assert np.array_equal(noisy.numpy(), ref)
    else:
        assert float((noisy - clean.cpu()).std()) > 0.0


@pytest.mark.parametrize("prec", PRECS)
def test_config1_full_size_step_properties(prec):
    """BASELINE config 1 (bs=64, 256x256x1): one full N2N step; per-image independence lets a
    single image be checked against the oracle at full resolution."""
    from image_denoising_amd import N2NTrainer
    from oracle import unet_ref

    net = _net(1, prec)
    g = torch.Generator(device="cpu").manual_seed(0)
    clean = F.interpolate(torch.rand(64, 1, 32, 32, generator=g), size=(256, 256),
                          mode="bilinear", align_corners=False).to(DEV)
    tr = N2NTrainer(net, seed=0)
    flat0 = net.flat_params.detach().cpu().clone()
    loss3 = tr.train_step(clean, epoch=1)
    torch.cuda.synchronize()
    l = loss3.cpu().numpy()
    assert np.isfinite(l).all() and l[0] > 0
    den0 = tr._bufs[next(iter(tr._bufs))]["den"][:2].cpu()
    noisy0 = tr._bufs[next(iter(tr._bufs))]["noisy"][:2].cpu()
    ref = unet_ref.forward(flat0, noisy0, 1, 1)
    # the no-grad pass defines den at the two pair pixels of every cell (what the loss reads)
    sel = _pair_mask(tr.last_rd[:2 * 128 * 128].cpu(), 2, 256, 256)
    assert rel_err(den0.numpy()[sel], ref.numpy()[sel]) < FP32_TOL
    assert torch.isfinite(tr.grad).all()


def _layer_errs(got, want, C=1):
    """per-layer max-norm relative error of two flat parameter-sized vectors"""
    from oracle.unet_ref import layer_table

    out, off = {}, 0
    for name_, ws, bl, _ in layer_table(C, C):
        n = int(np.prod(ws)) + bl
        out[name_] = rel_err(got[off:off + n], want[off:off + n])
        off += n
    return out


@pytest.fixture(scope="module")
def config1_oracle():
    """inputs of the headline-size step and the fp32 oracle's step on them (computed once for
    both arithmetics)"""
    from image_denoising_amd.arch_unet import reference_init
    from oracle import unet_ref

    N, H = 64, 256
    torch.manual_seed(0)
    flat0 = reference_init(1, 1, 48)
    g = torch.Generator(device="cpu").manual_seed(7)
    clean = F.interpolate(torch.rand(N, 1, 32, 32, generator=g), size=(H, H), mode="bilinear",
                          align_corners=False)
    noisy = (clean + (25.0 / 255.0) * torch.randn(clean.shape, generator=g)).float()
    rd = torch.randint(0, 8, (N * (H // 2) * (H // 2),), generator=g, dtype=torch.int64)
    r32 = unet_ref.n2n_step(flat0, noisy, rd.numpy().astype(np.uint8), 0.02)
    return dict(flat0=flat0, noisy=noisy, rd=rd, r32=r32)


@pytest.mark.parametrize("prec", PRECS)
def test_config1_full_size_step_vs_oracle(prec, config1_oracle):
    """The headline workload itself (BASELINE configs[1]: 64 x 1 x 256^2, reference init): one
    N2N step on the device and on the CPU oracle (unet_ref.n2n_step: torch autograd of the
    restatement, torch.optim.Adam; training_script.md:137-155, train.py:359-368) from the same
    noisy batch and the same rd_idx.
      * loss1, loss2 (Lambda-weighted regulariser) and loss within 1e-4 of the fp32 oracle;
      * den (the no-grad pass) at the two pair pixels of every cell of all 64 images within
        1e-4 of max |den| of the oracle's full forward;
      * the flat gradient per layer within 2e-5 of an fp64 restatement of the step's backward
        (sub1 forward, N2N loss on the device's den, autograd) that takes its LeakyReLU slopes
        and pool routing from the device's own saved activations of this step: only the
        rounding of the linear ops remains (as test_unet_unit_gain_fwd_bwd_vs_fp64).  Without
        that, any two fp32 forwards (the oracle's too: 1-4e-3 per layer at this size,
        tools/probes/r5_enc6.py) flip slopes at pre-activations within rounding of 0, so the
        free comparison against the fp32 oracle is only bounded loosely (1e-2);
      * the Adam update as test_n2n_step_vs_reference checks it (first-step updates are
        ~lr * sign(g): only gradients within rounding of zero may differ, by <= 2 lr)."""
    _full_size_step_vs_oracle(config1_oracle, 1, prec)


def _full_size_step_vs_oracle(o, C, prec):
    """shared body of the full-size step tests (configs[1] and configs[3]); see the docstring
    of test_config1_full_size_step_vs_oracle.  Beyond loss1 / loss it pins the regulariser
    loss2 (the only place the no-grad pass's den enters the step, training_script.md:150-152)
    and den itself at the pair pixels of EVERY image, both within 1e-4 of the fp32 oracle."""
    from image_denoising_amd import N2NTrainer
    from oracle import n2n_ref
    from oracle.unet_ref import forward

    N, _, H, W = o["noisy"].shape
    net = _net(C, prec)
    flat0 = o["flat0"]
    assert torch.equal(net.flat_params.detach().cpu(), flat0)
    tr = N2NTrainer(net, lr=3e-4, n_epoch=100, increase_ratio=2.0)
    lam = tr.lambda_for(1)
    assert lam == 0.02
    loss3 = tr.train_step(o["noisy"].to(DEV), epoch=1, rd_idx=o["rd"].to(torch.uint8).to(DEV),
                          noisy=o["noisy"].to(DEV)).cpu().numpy()
    grad = tr.grad.cpu().numpy()
    post = net.flat_params.detach().cpu().numpy()
    r32 = o["r32"]
    assert abs(loss3[0] - r32["loss1"]) <= FP32_TOL * r32["loss1"], (loss3, r32["loss1"])
    assert abs(loss3[1] - r32["loss2"]) <= FP32_TOL * r32["loss2"], (loss3, r32["loss2"])
    assert abs(loss3[2] - r32["loss"]) <= FP32_TOL * r32["loss"], (loss3, r32["loss"])
    b = tr._bufs[next(iter(tr._bufs))]
    # den at the two pair pixels of every cell of all N images (what the loss reads)
    sel = np.broadcast_to(_pair_mask(o["rd"], N, H, W), (N, C, H, W))
    den_dev, den_ref = b["den"].cpu().numpy()[sel], r32["den"].numpy()[sel]
    assert sel.sum() == N * C * H * W // 2
    assert np.abs(den_dev - den_ref).max() <= FP32_TOL * np.abs(den_ref).max()
    # fp64 backward of this step with the device's slopes and pool routing
    acts = _ws_activations(net, b["ws_grad"], N, H // 2, W // 2)
    m1, m2 = n2n_ref.masks_from_rd(o["rd"].numpy().astype(np.uint8))
    den = b["den"].cpu().double().numpy()
    exp_diff = torch.from_numpy(n2n_ref.generate_subimages(den, m1) -
                                n2n_ref.generate_subimages(den, m2))
    p64 = flat0.double().requires_grad_(True)
    y64 = forward(p64, r32["sub1"].double(), C, C, masks=acts)
    diff = y64 - r32["sub2"].double()
    (torch.mean(diff ** 2) + lam * torch.mean((diff - exp_diff) ** 2)).backward()
    e_dev = _layer_errs(grad, p64.grad.numpy(), C)
    worst = sorted(e_dev.items(), key=lambda kv: -kv[1])[:4]
    assert worst[0][1] < 2e-5, worst
    e_free = _layer_errs(grad, r32["grad"].numpy(), C)
    assert max(e_free.values()) < 1e-2, sorted(e_free.items(), key=lambda kv: -kv[1])[:4]
    upd, ref_upd = post - flat0.numpy(), r32["params"].numpy() - flat0.numpy()
    dd = np.abs(upd - ref_upd) > 1e-6
    assert dd.mean() < 2e-3, dd.mean()
    assert np.abs(upd - ref_upd).max() <= 6.1e-4  # never more than 2*lr apart


@pytest.fixture(scope="module")
def config3_oracle():
    """inputs of BASELINE configs[3]'s per-GPU step (32 x 3 x 256^2 RGB, reference init) and the
    fp32 oracle's step on them"""
    from image_denoising_amd.arch_unet import reference_init
    from oracle import unet_ref

    N, C, H = 32, 3, 256
    torch.manual_seed(0)
    flat0 = reference_init(C, C, 48)
    g = torch.Generator(device="cpu").manual_seed(9)
    clean = F.interpolate(torch.rand(N, C, 32, 32, generator=g), size=(H, H), mode="bilinear",
                          align_corners=False)
    noisy = (clean + (25.0 / 255.0) * torch.randn(clean.shape, generator=g)).float()
    rd = torch.randint(0, 8, (N * (H // 2) * (H // 2),), generator=g, dtype=torch.int64)
    r32 = unet_ref.n2n_step(flat0, noisy, rd.numpy().astype(np.uint8), 0.02, in_nc=C, out_nc=C)
    return dict(flat0=flat0, noisy=noisy, rd=rd, r32=r32)


@pytest.mark.parametrize("prec", PRECS)
def test_config3_full_size_step_vs_oracle(prec, config3_oracle):
    """BASELINE configs[3]'s per-GPU step at full size (32 x 3 x 256^2 RGB, reference init)
    against the fp32 oracle: loss1, loss2, loss, den at every pair pixel of all 32 images, the
    per-layer gradient against the fp64 restatement with the device's slopes / routing, and
    the Adam update (as test_config1_full_size_step_vs_oracle)."""
    _full_size_step_vs_oracle(config3_oracle, 3, prec)


@pytest.mark.parametrize("prec", PRECS)
def test_config3_full_size_rgb_step_properties(prec):
    """BASELINE configs[3] at full size: 32 x 3 x 256^2 RGB patches, one N2N step.  Images are
    independent: image 0's denoised output at the pair pixels (all the step reads) is checked
    against the oracle at full resolution."""
    from image_denoising_amd import N2NTrainer
    from oracle import unet_ref

    net = _net(3, prec)
    g = torch.Generator(device="cpu").manual_seed(5)
    clean = F.interpolate(torch.rand(32, 3, 32, 32, generator=g), size=(256, 256),
                          mode="bilinear", align_corners=False).to(DEV)
    tr = N2NTrainer(net, seed=1)
    flat0 = net.flat_params.detach().cpu().clone()
    loss3 = tr.train_step(clean, epoch=1)
    torch.cuda.synchronize()
    l = loss3.cpu().numpy()
    assert np.isfinite(l).all() and l[0] > 0
    assert bool(torch.isfinite(tr.grad).all()) and float(tr.grad.abs().max()) > 0
    b = tr._bufs[next(iter(tr._bufs))]
    den0, noisy0 = b["den"][:1].cpu(), b["noisy"][:1].cpu()
    with torch.no_grad():
        ref = unet_ref.forward(flat0, noisy0, 3, 3)
    sel = np.broadcast_to(_pair_mask(tr.last_rd[:128 * 128].cpu(), 1, 256, 256), (1, 3, 256, 256))
    assert rel_err(den0.numpy()[sel], ref.numpy()[sel]) < FP32_TOL


@pytest.mark.parametrize("C", [1, 3])
def test_structure_step_vs_oracle(C):
    """train.py:355-368 (Structure_loss step: two grad forwards, one backward, Adam) through
    StructureTrainer vs the oracle: torch autograd of the fp32 CPU UNet restatement with the
    same loss, and torch.optim.Adam."""
    from image_denoising_amd import StructureTrainer
    from oracle.unet_ref import forward

    net = _net(C)
    flat0 = net.flat_params.detach().cpu().clone()
    g = torch.Generator().manual_seed(11)
    clean = torch.rand(2, C, 64, 64, generator=g)
    noisy = clean + 0.1 * torch.randn(2, C, 64, 64, generator=g)
    tr = StructureTrainer(net, lr=3e-4, n_epoch=100)
    loss5 = tr.train_step(clean.to(DEV), noisy.to(DEV), epoch=1).cpu().numpy()
    grad = tr.grad.cpu().numpy()
    # oracle
    p = flat0.clone().requires_grad_(True)
    pred, pred2 = forward(p, noisy, C, C), forward(p, clean, C, C)
    l1 = torch.nn.L1Loss()
    parts = [l1(pred, clean), l1(pred2[:, :, 1:], pred2[:, :, :-1]),
             l1(pred2[..., 1:], pred2[..., :-1]), l1(pred2, clean)]
    loss = parts[0] + 0.5 * (parts[1] + parts[2]) / 2 + 0.5 * parts[3]
    loss.backward()
    want = [float(t) for t in parts] + [float(loss)]
    for got, w in zip(loss5, want):
        assert abs(got - w) <= FP32_TOL * abs(w), (loss5, want)
    assert rel_err(grad, p.grad.numpy()) < 1e-3
    q = flat0.clone().requires_grad_(True)
    opt = torch.optim.Adam([q], lr=3e-4)
    q.grad = p.grad.clone()
    opt.step()
    upd = net.flat_params.detach().cpu().numpy() - flat0.numpy()
    ref_upd = (q.detach() - flat0).numpy()
    bad = np.abs(upd - ref_upd) > 1e-6  # Adam's first step is ~lr*sign(g): tiny-g sign flips
    assert bad.mean() < 2e-3, bad.mean()
    assert np.abs(upd - ref_upd).max() <= 6.1e-4


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("C", [1, 3])
def test_n2n_trajectory_vs_oracle(C, prec):
    """SURVEY §8d eval parity: several N2N steps (train.py:356-368) with the same inputs and
    rd_idx stream on the HIP path and on the oracle (torch.optim.Adam state carried across
    steps), then the denoised image of a held-out input (evaluation.py:74) compared at the
    fp32 tolerance.  Adam's first updates are ~lr in size whatever the gradient, so a parameter
    whose gradient is within rounding of zero can move +lr on one side and -lr on the other;
    the check is on the losses and the network output, as the metric is."""
    from image_denoising_amd import N2NTrainer
    from image_denoising_amd.arch_unet import reference_init
    from oracle import unet_ref

    steps, N, H = 4, 2, 64
    net = _net(C, prec)
    torch.manual_seed(0)
    flat = reference_init(C, C, 48)
    assert torch.equal(net.flat_params.detach().cpu(), flat)
    g = torch.Generator(device="cpu").manual_seed(5)
    clean = F.interpolate(torch.rand(N, C, 16, 16, generator=g), size=(H, H), mode="bilinear",
                          align_corners=False)
    tr = N2NTrainer(net, lr=3e-4, n_epoch=100, increase_ratio=2.0)
    state = None
    for s in range(steps):
        noisy = (clean + (25.0 / 255.0) * torch.randn(clean.shape, generator=g)).float()
        rd = torch.randint(0, 8, (N * (H // 2) * (H // 2),), generator=g, dtype=torch.int64)
        l_gpu = tr.train_step(noisy.to(DEV), epoch=1, rd_idx=rd.to(DEV).to(torch.uint8),
                              noisy=noisy.to(DEV)).cpu().numpy()
        r = unet_ref.n2n_step(flat, noisy, rd.numpy().astype(np.uint8), 0.02, adam_state=state,
                             in_nc=C, out_nc=C)
        flat, state = r["params"], r["adam_state"]
        assert abs(l_gpu[0] - r["loss1"]) <= FP32_TOL * r["loss1"], (s, l_gpu, r["loss1"])
        assert abs(l_gpu[2] - r["loss"]) <= FP32_TOL * r["loss"], (s, l_gpu, r["loss"])
    x = (clean + (25.0 / 255.0) * torch.randn(clean.shape, generator=g)).float()
    with torch.no_grad():
        y = net(x.to(DEV)).cpu()
    y_ref = unet_ref.forward(flat, x, C, C)
    assert rel_err(y.numpy(), y_ref.numpy()) < FP32_TOL
