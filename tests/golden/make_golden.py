"""Generates tests/golden/*.npz from the REFERENCE implementation (build container only).

Run:  python tests/golden/make_golden.py [/root/reference]

What it executes from the reference (read from its source tree, nothing is copied into this
repo):
  - arch_unet.UNet and util.Structure_loss, imported as modules;
  - train.py's space_to_depth / generate_mask_pair / generate_subimages (train.py:134-190),
    AST-extracted and exec'd with a CPU stand-in for get_generator (train.py:56-61 hard-codes
    device="cuda" and reads a never-initialised global, train.py:43);
  - utils_eval.calculate_psnr (utils_eval.py:49-53), AST-extracted (the module imports cv2,
    which is absent here).
The fixtures are data only (inputs and expected outputs); the GPU box never needs the reference.
"""
from __future__ import annotations

import ast
import hashlib
import os
import sys

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "/root/reference"


def extract(path: str, names: list[str], ns: dict) -> dict:
    src = open(path).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    missing = set(names) - {n.name for n in keep}
    assert not missing, missing
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
    return ns


def cpu_generator_namespace():
    state = {"counter": 0}

    def get_generator():  # train.py:56-61 on the CPU
        state["counter"] += 1
        g = torch.Generator(device="cpu")
        g.manual_seed(state["counter"])
        return g

    return {"torch": torch, "get_generator": get_generator}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def flat_params(net) -> np.ndarray:
    return torch.cat([v.reshape(-1) for v in net.state_dict().values()]).numpy().astype(np.float32)


def main():
    sys.path.insert(0, REF)
    import arch_unet  # noqa: E402
    import util  # noqa: E402

    ns = extract(os.path.join(REF, "train.py"),
                 ["space_to_depth", "generate_mask_pair", "generate_subimages"],
                 cpu_generator_namespace())

    # ---- 1. sub-sampler ------------------------------------------------------------------
    fx = {}
    img = torch.arange(2 * 3 * 8 * 8, dtype=torch.float32).reshape(2, 3, 8, 8)
    m1, m2 = ns["generate_mask_pair"](img)
    fx["a_img"] = img.numpy()
    fx["a_mask1"], fx["a_mask2"] = m1.numpy(), m2.numpy()
    fx["a_sub1"] = ns["generate_subimages"](img, m1).numpy()
    fx["a_sub2"] = ns["generate_subimages"](img, m2).numpy()
    # rd_idx recovered from the masks (one-hot per cell): pair table lookup
    pairs = [[0, 1], [0, 2], [1, 3], [2, 3], [1, 0], [2, 0], [3, 1], [3, 2]]
    def rd_from(m1, m2):
        k1 = m1.reshape(-1, 4).argmax(1)
        k2 = m2.reshape(-1, 4).argmax(1)
        lut = {tuple(p): i for i, p in enumerate(pairs)}
        return np.array([lut[(a, b)] for a, b in zip(k1.tolist(), k2.tolist())], dtype=np.uint8)
    fx["a_rd"] = rd_from(m1.numpy(), m2.numpy())
    g = torch.Generator().manual_seed(5)
    img = torch.rand(4, 1, 64, 64, generator=g)
    m1, m2 = ns["generate_mask_pair"](img)
    fx["b_img"] = img.numpy()
    fx["b_rd"] = rd_from(m1.numpy(), m2.numpy())
    fx["b_sub1"] = ns["generate_subimages"](img, m1).numpy()
    fx["b_sub2"] = ns["generate_subimages"](img, m2).numpy()
    # ragged-looking but valid: non-square, C=3
    img = torch.rand(1, 3, 6, 10, generator=g)
    m1, m2 = ns["generate_mask_pair"](img)
    fx["c_img"] = img.numpy()
    fx["c_rd"] = rd_from(m1.numpy(), m2.numpy())
    fx["c_sub1"] = ns["generate_subimages"](img, m1).numpy()
    fx["c_sub2"] = ns["generate_subimages"](img, m2).numpy()
    np.savez_compressed(os.path.join(OUT, "subsampler.npz"), **fx)

    unet_main()

    # ---- 3. one N2N step (training_script.md:137-155) with torch.optim.Adam ---------------
    torch.manual_seed(0)
    net = arch_unet.UNet(in_nc=1, out_nc=1, n_feature=48)
    g = torch.Generator().manual_seed(2)
    clean = torch.nn.functional.interpolate(torch.rand(2, 1, 16, 16, generator=g), size=(64, 64),
                                            mode="bilinear", align_corners=False)
    noisy = clean + torch.normal(0.0, 25.0 / 255.0, size=clean.shape, generator=g)
    ns2 = extract(os.path.join(REF, "train.py"),
                  ["space_to_depth", "generate_mask_pair", "generate_subimages"],
                  cpu_generator_namespace())
    optimizer = torch.optim.Adam(net.parameters(), lr=3e-4)
    epoch, n_epoch, ratio = 1, 100, 2.0
    mask1, mask2 = ns2["generate_mask_pair"](noisy)
    noisy_sub1 = ns2["generate_subimages"](noisy, mask1)
    noisy_sub2 = ns2["generate_subimages"](noisy, mask2)
    with torch.no_grad():
        noisy_denoised = net(noisy)
    noisy_sub1_denoised = ns2["generate_subimages"](noisy_denoised, mask1)
    noisy_sub2_denoised = ns2["generate_subimages"](noisy_denoised, mask2)
    noisy_output = net(noisy_sub1)
    noisy_output.retain_grad()
    Lambda = epoch / n_epoch * ratio
    diff = noisy_output - noisy_sub2
    exp_diff = noisy_sub1_denoised - noisy_sub2_denoised
    loss1 = torch.mean(diff ** 2)
    loss2 = Lambda * torch.mean((diff - exp_diff) ** 2)
    loss_all = loss1 + loss2
    optimizer.zero_grad()
    loss_all.backward()
    grad = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).numpy()
    pre = flat_params(net)
    optimizer.step()
    post = flat_params(net)
    idx = np.random.default_rng(1).choice(post.size, 16384, replace=False)
    np.savez_compressed(
        os.path.join(OUT, "n2n_step.npz"), noisy=noisy.numpy(), rd=rd_from(mask1.numpy(), mask2.numpy()),
        lam=np.float32(Lambda), loss1=np.float32(loss1.item()), loss2=np.float32(loss2.item()),
        loss=np.float32(loss_all.item()), dout=noisy_output.grad.numpy(),
        den=noisy_denoised.numpy(), out=noisy_output.detach().numpy(),
        grad_idx=idx, grad_sample=grad[idx], grad_norm=np.float64(np.linalg.norm(grad)),
        post_idx=idx, post_sample=post[idx], post_minus_pre_sum=np.float64((post.astype(np.float64) - pre).sum()),
        pre_sha=np.array(sha(pre)))

    # ---- 4. Structure_loss (util.py:41-70) -------------------------------------------------
    g = torch.Generator().manual_seed(3)
    pred = torch.rand(2, 1, 16, 16, generator=g).requires_grad_(True)
    pred2 = torch.rand(2, 1, 16, 16, generator=g).requires_grad_(True)
    tgt = torch.rand(2, 1, 16, 16, generator=g)
    crit = util.Structure_loss()
    L = crit(pred, pred2, tgt)
    L.backward()
    np.savez_compressed(os.path.join(OUT, "structure_loss.npz"), pred=pred.detach().numpy(),
                        pred2=pred2.detach().numpy(), target=tgt.numpy(), loss=np.float32(L.item()),
                        dpred=pred.grad.numpy(), dpred2=pred2.grad.numpy())

    # ---- 5. PSNR (utils_eval.py:49-53) known answers ----------------------------------------
    nsp = extract(os.path.join(REF, "utils_eval.py"), ["calculate_psnr"], {"np": np})
    rng = np.random.default_rng(4)
    a = rng.integers(0, 256, (2, 48, 40), dtype=np.uint8)
    b = np.clip(a.astype(np.int32) + rng.integers(-9, 10, a.shape), 0, 255).astype(np.uint8)
    psnr = np.array([nsp["calculate_psnr"](a[i], b[i]) for i in range(2)])
    np.savez_compressed(os.path.join(OUT, "eval_psnr.npz"), a=a, b=b, psnr=psnr)
    print("golden fixtures written to", OUT)


def unet_main():
    """arch_unet.UNet (imported): init, forward, dL/dx and parameter gradients of mean(y^2), and
    the state_dict key names / shapes (the checkpoint contract, evaluation.py:52-53)."""
    sys.path.insert(0, REF)
    import arch_unet  # noqa: E402

    for C, N, path in ((1, 2, "unet_c1.npz"), (3, 1, "unet_c3.npz")):
        torch.manual_seed(0)
        net = arch_unet.UNet(in_nc=C, out_nc=C, n_feature=48)
        flat = flat_params(net)
        x = torch.rand(N, C, 64, 64, generator=torch.Generator().manual_seed(1))
        x.requires_grad_(True)
        y = net(x)
        loss = (y ** 2).mean()
        loss.backward()
        grad = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).numpy()
        fx = dict(x=x.detach().numpy(), y=y.detach().numpy(), loss=np.float32(loss.item()),
                  dx=x.grad.numpy(),
                  params_sha=np.array(sha(flat)), params_sum=np.float64(flat.astype(np.float64).sum()),
                  params_head=flat[:64],
                  keys=np.array(list(net.state_dict().keys())),
                  key_shapes=np.array([list(v.shape) + [0] * (4 - v.dim())
                                       for v in net.state_dict().values()], dtype=np.int64))
        if C == 1:
            fx["grad"] = grad
        else:
            idx = np.random.default_rng(0).choice(grad.size, 8192, replace=False)
            fx["grad_idx"], fx["grad_sample"] = idx, grad[idx]
        fx["grad_norms"] = np.array([np.linalg.norm(p.grad.numpy()) for p in net.parameters()])
        np.savez_compressed(os.path.join(OUT, path), **fx)
    print("UNet fixtures written to", OUT)


def adapter_main():
    """adapter.py OutputAdapter / DenoiserWithAdapter (imported) and finetune.py's gradient /
    gradient_loss (AST-extracted: finetune.py imports torchvision, absent here)."""
    sys.path.insert(0, REF)
    import adapter  # noqa: E402
    import arch_unet  # noqa: E402

    ft = extract(os.path.join(REF, "finetune.py"), ["gradient", "gradient_loss"],
                 {"torch": torch, "F": torch.nn.functional})
    fx = {}
    # ---- 6a. OutputAdapter alone, C = 1 and 3: output + parameter grads of the finetune loss
    for C in (1, 3):
        torch.manual_seed(10 + C)
        ad = adapter.OutputAdapter(in_channels=C, hidden_channels=16)
        g = torch.Generator().manual_seed(20 + C)
        noisy = torch.rand(2, C, 24, 40, generator=g)
        base = torch.rand(2, C, 24, 40, generator=g)
        clean = torch.rand(2, C, 24, 40, generator=g)
        out = ad(noisy, base)
        l1 = torch.nn.functional.l1_loss(out, clean)
        lg = ft["gradient_loss"](out, clean)
        loss = l1 + 0.1 * lg
        loss.backward()
        k = f"c{C}_"
        fx[k + "params"] = torch.cat([v.reshape(-1) for v in ad.state_dict().values()]).numpy()
        fx[k + "noisy"], fx[k + "base"], fx[k + "clean"] = noisy.numpy(), base.numpy(), clean.numpy()
        fx[k + "out"] = out.detach().numpy()
        fx[k + "loss"] = np.array([l1.item(), lg.item(), loss.item()], np.float32)
        fx[k + "grad"] = torch.cat([p.grad.reshape(-1) for p in ad.parameters()]).numpy()
    # ---- 6b. one finetune.py:269-289 step, DenoiserWithAdapter(UNet base), Adam lr 1e-4
    torch.manual_seed(0)
    base = arch_unet.UNet(in_nc=1, out_nc=1, n_feature=48)
    torch.manual_seed(1)
    model = adapter.DenoiserWithAdapter(base, in_channels=1, hidden_channels=16)
    g = torch.Generator().manual_seed(30)
    clean = torch.rand(2, 1, 64, 64, generator=g)
    noisy = clean + 0.1 * torch.randn(2, 1, 64, 64, generator=g)
    opt = torch.optim.Adam(filter(lambda p: p.requires_grad, model.parameters()), lr=1e-4)
    opt.zero_grad()
    pred = model(noisy)
    l1 = torch.nn.functional.l1_loss(pred, clean)
    lg = ft["gradient_loss"](pred, clean)
    loss = l1 + 0.1 * lg
    loss.backward()
    grad = torch.cat([p.grad.reshape(-1) for p in model.adapter.parameters()]).numpy()
    pre = torch.cat([p.detach().reshape(-1) for p in model.adapter.parameters()]).numpy().copy()
    opt.step()
    post = torch.cat([p.detach().reshape(-1) for p in model.adapter.parameters()]).numpy()
    fx.update(step_noisy=noisy.numpy(), step_clean=clean.numpy(), step_pred=pred.detach().numpy(),
              step_loss=np.array([l1.item(), lg.item(), loss.item()], np.float32),
              step_grad=grad, step_pre=pre, step_post=post,
              step_base_sha=np.array(sha(flat_params(base))))
    np.savez_compressed(os.path.join(OUT, "adapter.npz"), **fx)
    print("adapter fixtures written to", OUT)


def iunet_main():
    """arch_unet.ImprovedUNet (imported): init, forward, parameter gradients of a squared error."""
    sys.path.insert(0, REF)
    import arch_unet  # noqa: E402

    for C, N, S, path in ((1, 2, 32, "iunet_c1.npz"), (3, 1, 32, "iunet_c3.npz")):
        torch.manual_seed(0)
        net = arch_unet.ImprovedUNet(in_nc=C, out_nc=C, n_feature=48)
        flat = flat_params(net)
        g = torch.Generator().manual_seed(1)
        x = torch.rand(N, C, S, S, generator=g)
        t = torch.rand(N, C, S, S, generator=g)
        y = net(x)
        loss = ((y - t) ** 2).mean()
        loss.backward()
        grad = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).numpy()
        idx = np.random.default_rng(0).choice(grad.size, 16384, replace=False)
        np.savez_compressed(
            os.path.join(OUT, path), x=x.numpy(), t=t.numpy(), y=y.detach().numpy(),
            loss=np.float32(loss.item()), params_sha=np.array(sha(flat)),
            params_count=np.int64(flat.size), grad_idx=idx, grad_sample=grad[idx],
            grad_norms=np.array([np.linalg.norm(p.grad.numpy()) for p in net.parameters()]),
            keys=np.array(list(net.state_dict().keys())))
    print("ImprovedUNet fixtures written to", OUT)


if __name__ == "__main__":
    if "--only" in sys.argv:
        {"adapter": adapter_main, "iunet": iunet_main, "unet": unet_main}[sys.argv[sys.argv.index("--only") + 1]]()
    else:
        main()
        adapter_main()
        iunet_main()
