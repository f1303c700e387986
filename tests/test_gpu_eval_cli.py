"""The evaluation CLIs end to end on the HIP path (BASELINE's "eval PSNR vs ref" half):
evaluation.py (evaluation.py:19-114: --log_name UNET and the reference's default UNetImproved)
and evaluation_adapter.py (evaluation_adapter.py:83-166) over a two-image temporary dataset,
against the CPU oracle's denoised images and metrics with the same checkpoint.  Needs an MI355X."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
H, W = 96, 128  # multiples of 32 (UNet) and 16 (ImprovedUNet)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _dataset(root):
    from PIL import Image

    rng = np.random.default_rng(21)
    clean, noisy = [], []
    for d in ("clean", "noise"):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    for i in range(2):
        yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
        c = np.clip(128 + 90 * np.sin(3 * xx + 2 * yy + i), 0, 255).astype(np.uint8)
        n = np.clip(c.astype(int) + rng.integers(-25, 26, c.shape), 0, 255).astype(np.uint8)
        Image.fromarray(c).save(os.path.join(root, "clean", f"img{i}.png"))
        Image.fromarray(n).save(os.path.join(root, "noise", f"img{i}.png"))
        clean.append(c)
        noisy.append(n)
    return clean, noisy


def _scaled(net, f):
    torch.manual_seed(0)
    with torch.no_grad():  # larger-than-init weights so the output is not ~constant
        for name, p in net.named_parameters():
            if name.endswith("weight"):
                p.mul_(f)
    return net


def _oracle_metrics(preds, clean):
    from oracle import eval_ref

    ps, ss = [], []
    for p, c in zip(preds, clean):
        q = eval_ref.quantize_full(p)
        ps.append(eval_ref.psnr(q, c))
        ss.append(eval_ref.calculate_ssim(q, c))
    return float(np.mean(ps)), float(np.mean(ss))


def _read_metrics(path):
    vals = {}
    for line in open(path):
        k, v = line.rsplit(":", 1)
        vals[k.strip()] = float(v)
    return vals


@pytest.mark.parametrize("log_name", ["UNET", "UNetImproved"])
def test_evaluation_cli_matches_oracle(tmp_path, log_name):
    from image_denoising_amd import UNet, evaluation
    from image_denoising_amd.checkpoint import save_checkpoint
    from image_denoising_amd.improved_unet import ImprovedUNet
    from oracle import iunet_ref, unet_ref

    torch.manual_seed(0)
    if log_name == "UNET":
        net, fwd, f = UNet(1, 1, 48), unet_ref.forward, 8.0
    else:
        net, fwd, f = ImprovedUNet(1, 1, 48), iunet_ref.forward, 1.5
    _scaled(net, f)
    ck = save_checkpoint(net, str(tmp_path / "ck.pth"), data_parallel=True)
    clean, noisy = _dataset(str(tmp_path / "data"))
    out = str(tmp_path / "out")
    res = evaluation.main(["--data_dir", str(tmp_path / "data"), "--checkpoint", ck,
                           "--save_dir", out, "--log_name", log_name])
    flat = net.flat_params.detach().cpu()
    preds, l1s = [], []
    with torch.no_grad():
        for n in noisy:
            x = torch.from_numpy(n.astype(np.float32) / 255.0)[None, None]
            y = fwd(flat, x, 1, 1)
            preds.append(y.numpy()[0, 0])
            l1s.append(float((y - x).abs().mean()))
    psnr_w, ssim_w = _oracle_metrics(preds, clean)
    # single-pixel rounding-boundary flips of the uint8 quantisation move PSNR by < 1e-3 dB here
    assert res["avg_psnr"] == pytest.approx(psnr_w, abs=2e-3)
    assert res["avg_ssim"] == pytest.approx(ssim_w, abs=1e-4)
    assert res["avg_l1"] == pytest.approx(float(np.mean(l1s)), rel=1e-4)
    m = _read_metrics(os.path.join(out, "metrics.txt"))
    assert m["Average PSNR"] == round(res["avg_psnr"], 2)
    assert m["Average SSIM"] == round(res["avg_ssim"], 4)
    assert m["Average L1 Loss"] == round(res["avg_l1"], 6)


def test_evaluation_cli_rejects_out_of_scope_networks(tmp_path):
    from image_denoising_amd import evaluation

    for name in ("UNET_blindspot", "RESNET", "foo"):
        with pytest.raises(SystemExit):
            evaluation.main(["--data_dir", str(tmp_path), "--checkpoint", "x.pth", "--log_name", name])


def test_evaluation_adapter_cli_matches_oracle(tmp_path):
    from image_denoising_amd import UNet, evaluation_adapter
    from image_denoising_amd.adapter import DenoiserWithAdapter
    from oracle import adapter_ref, eval_ref, unet_ref

    torch.manual_seed(0)
    base = _scaled(UNet(1, 1, 48), 8.0)
    model = DenoiserWithAdapter(base, in_channels=1, hidden_channels=16)
    with torch.no_grad():
        g = torch.Generator().manual_seed(3)
        model.adapter.flat_params.copy_(0.05 * torch.randn(model.adapter.flat_params.shape, generator=g))
    sd = {"module." + k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    ck = str(tmp_path / "epoch_adapter_001.pth")
    torch.save(sd, ck)
    clean, noisy = _dataset(str(tmp_path / "data"))
    out = str(tmp_path / "out")
    res = evaluation_adapter.main(["--data_dir", str(tmp_path / "data"), "--ckpt", ck, "--arch", "UNet",
                                   "--save_dir", out])
    bflat, aflat = base.flat_params.detach().cpu(), model.adapter.flat_params.detach().cpu()
    for i, (n, c) in enumerate(zip(noisy, clean)):
        x = torch.from_numpy(n.astype(np.float32) / 255.0)[None, None]
        with torch.no_grad():
            y = adapter_ref.adapter_forward(aflat, x, unet_ref.forward(bflat, x, 1, 1))
        q = np.clip(y.numpy()[0, 0] * np.float32(255.0) + np.float32(0.5), 0, 255).astype(np.uint8)
        assert res["psnr"][i] == pytest.approx(eval_ref.psnr(q, c), abs=2e-3)
        assert os.path.exists(os.path.join(out, f"img{i}_denoised.png"))
