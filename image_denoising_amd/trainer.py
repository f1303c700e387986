"""The N2N training step (training_script.md:128-155 with train.py's sub-sampler), fused on
the HIP path with no host synchronisation:

    noisy  = clean + sigma*N(0,1)                     dn_add_gauss_noise   (train.py:84-101)
             (or Poisson(lam clean) / lam             dn_add_poisson_noise (train.py:102-111))
    sub1, sub2, rd = neighbour sub-sample(noisy)      dn_n2n_subsample     (train.py:141-190)
    den    = UNet(noisy)            [no grad]         dn_unet_forward      (arch_unet.py:194)
    out    = UNet(sub1)             [saved]           dn_unet_forward
    loss, dout = N2N loss(out, sub2, den[rd])         dn_n2n_loss          (training_script.md:148-153)
    dW     = backward(dout)                           dn_unet_backward
    [data parallel: one RCCL all-reduce(sum) of the flat dW]
    Adam(W, dW / world)                               dn_adam_step         (train.py:332, :368)

Data parallelism: one process per GPU; rank r owns patches [r*B, (r+1)*B) of the global batch.
The Philox streams are keyed on GLOBAL element/cell indices and the step number, so the
noise and the mask pair of a patch do not depend on the world size.
"""
from __future__ import annotations

import os

import torch

from . import _lib
from . import dist as dp
from .arch_unet import UNet
from .n2n import AugmentNoise, n2n_loss, n2n_subsample
from .optim import FlatAdam, lr_at_epoch
from .util import structure_loss_into


class N2NTrainer:
    def __init__(self, net: UNet, lr: float = 3e-4, n_epoch: int = 100,
                 increase_ratio: float = 2.0, gamma: float = 0.5, noise_std: float = 25.0 / 255.0,
                 seed: int = 0, distributed: bool | None = None, noise_style: str | None = None):
        """noise_style: a train.py --noisetype ('gauss25', 'gauss5_50', 'poisson30',
        'poisson5_50'); None = Gaussian of std noise_std.  Range styles draw one value per image
        of the GLOBAL batch (seeded by the step), so a rank's shard sees the same values as the
        single-process run."""
        self.net = net
        self.base_lr = lr
        self.n_epoch = n_epoch
        self.increase_ratio = increase_ratio
        self.gamma = gamma
        self.noise_std = noise_std
        self.noise = AugmentNoise(noise_style) if noise_style else None
        self.seed = seed
        self.distributed = dp.require_group(distributed)
        self.world, self.rank = dp.world_and_rank() if self.distributed else (1, 0)
        if self.distributed:  # identical replicas: broadcast rank 0's initial weights
            dp.broadcast_params(net.flat_params)
        self.opt = FlatAdam(net.flat_params, lr=lr)
        self.grad = torch.zeros_like(net.flat_params)
        self.global_step = 0
        self._bufs = {}
        # the overlapped all-reduce needs the split backward (arch_unet.UNet); other nets
        # (ImprovedUNet) take the one all-reduce after the whole backward
        self._overlap = (os.environ.get("DN_AR_OVERLAP", "1") != "0"
                         and hasattr(net, "_run_backward_split") and hasattr(net, "tail_begin"))
        self._tail_begin = net.tail_begin() if self.distributed and self._overlap else 0

    @staticmethod
    def _comm_stream(device):
        """the stream the early gradient bucket's all-reduce is enqueued on"""
        if torch.device(device).type != "cuda":
            return None
        return dp.step_stream("comm", device)

    def _backward(self, dout, ws, N, h, w, ev):
        if ev is None:
            self.net._run_backward(dout, self.grad, ws, N, h, w)
        else:
            self.net._run_backward_split(dout, self.grad, ws, N, h, w, ev)

    @staticmethod
    def _side_stream(device):
        if os.environ.get("DN_STEP_STREAMS", "1") == "0" or torch.device(device).type != "cuda":
            return None
        return dp.step_stream("side", device)

    def lambda_for(self, epoch: int) -> float:
        # training_script.md:148 Lambda = epoch / n_epoch * ratio
        return epoch / self.n_epoch * self.increase_ratio

    def _buffers(self, N, C, H, W, device):
        key = (N, C, H, W, device)
        b = self._bufs.get(key)
        if b is None:
            h, w = H // 2, W // 2
            f = dict(dtype=torch.float32, device=device)
            b = dict(
                noisy=torch.empty((N, C, H, W), **f),
                den=torch.empty((N, self.net.out_nc, H, W), **f),
                out=torch.empty((N, self.net.out_nc, h, w), **f),
                ws_den=self.net._workspace(N, H, W, with_backward=False, fresh=True),
                ws_grad=self.net._workspace(N, h, w, with_backward=True, fresh=True),
            )
            self._bufs = {key: b}
        return b

    def train_step(self, clean: torch.Tensor, epoch: int = 1, rd_idx: torch.Tensor | None = None,
                   noisy: torch.Tensor | None = None) -> torch.Tensor:
        """One N2N step on this rank's local batch. Returns loss3 = [loss1, loss2, loss_all]
        (device tensor; read it only when needed — reading syncs the host)."""
        clean = clean.contiguous()
        N, C, H, W = clean.shape
        if C != self.net.in_nc or self.net.in_nc != self.net.out_nc:
            raise ValueError("N2N needs in_nc == out_nc == input channels")
        b = self._buffers(N, C, H, W, clean.device)
        stream = _lib.stream_of(clean)
        step = self.global_step
        elem_base, cell_base = dp.shard_bases(self.rank, N, C, H, W)
        if noisy is None:
            noisy = b["noisy"]
            fn, val, per_img = "dn_add_gauss_noise", float(self.noise_std), None
            if self.noise is not None:
                if not self.noise.style.startswith("gauss"):
                    fn = "dn_add_poisson_noise"
                val = float(self.noise.params[0])
                if self.noise.style.endswith("_range"):
                    lo, hi = self.noise.params
                    g = torch.Generator(device="cpu").manual_seed(self.seed * 1000003 + step)
                    allv = torch.rand(N * self.world, generator=g) * (hi - lo) + lo
                    per_img = allv[self.rank * N:(self.rank + 1) * N].to(clean.device)
            _lib.call(fn, _lib.ptr(clean), N, C * H * W, val, _lib.ptr(per_img), self.seed, 2 * step,
                      elem_base, _lib.ptr(noisy), stream)
        else:
            noisy = noisy.contiguous()
        sub1, sub2, rd = n2n_subsample(noisy, rd_idx, seed=self.seed + 1, offset=2 * step + 1,
                                       cell_base=cell_base)
        self.last_rd = rd  # the step's per-cell pair choices (den is defined at those pixels)
        # no-grad full-resolution pass (training_script.md:141-142); the loss reads the denoised
        # image at the rd pair pixels only, so only those are produced (dn_unet_forward_n2n)
        # It runs on a second stream beside the gradient pass's forward (separate workspaces,
        # both only read the parameters); the loss waits for both.  DN_STEP_STREAMS=0: one stream.
        side = self._side_stream(clean.device)
        main = torch.cuda.current_stream(clean.device) if side is not None else None
        if side is not None:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self.net._run_forward_n2n(noisy, b["den"], b["ws_den"], rd)
        else:
            self.net._run_forward_n2n(noisy, b["den"], b["ws_den"], rd)
        # gradient pass at half resolution (training_script.md:146)
        self.net._run_forward(sub1, b["out"], b["ws_grad"])
        if side is not None:
            main.wait_stream(side)
        loss3, dout = n2n_loss(b["out"], sub2, b["den"], rd, self.lambda_for(epoch))
        # RCCL all-reduce(sum) over xGMI; 1/world folded into Adam.  Data-parallel: two buckets,
        # the decoder + head one overlapping the encoder's backward (DN_AR_OVERLAP=0: one
        # all-reduce after the whole backward)
        if self.distributed and self._overlap:
            scale = dp.allreduce_grads_split(
                self.grad, self._tail_begin,
                lambda ev: self._backward(dout, b["ws_grad"], N, H // 2, W // 2, ev),
                self._comm_stream(clean.device))
        else:
            self.net._run_backward(dout, self.grad, b["ws_grad"], N, H // 2, W // 2)
            scale = dp.allreduce_grads(self.grad) if self.distributed else 1.0
        self.opt.lr = lr_at_epoch(epoch, self.base_lr, self.n_epoch, self.gamma)
        self.opt.step(self.grad, grad_scale=scale)
        self.global_step += 1
        return loss3


class StructureTrainer:
    """The step of the reference's own train.py loop (train.py:355-368), fused:

        pred, pred2 = UNet([noisy; clean])  [saved]   dn_unet_forward   (train.py:361-362)
        loss5, dpred, dpred2 = Structure_loss(pred, pred2, clean)
                                                      dn_structure_loss (util.py:56-70)
        dW = backward([dpred; dpred2])                dn_unet_backward
        [data parallel: one RCCL all-reduce(sum) of dW]
        Adam(W, dW / world)                           dn_adam_step      (train.py:368)

    `network(noisy)` and `network(clean)` share the weights, so they run as ONE forward and ONE
    backward over the 2N batch [noisy; clean]: the weight gradient of a batch is the sum over its
    images, i.e. dW(pred) + dW(pred2) exactly as autograd forms it in the reference, with half
    the launches and every small-level launch at twice the occupancy.

    Inputs are device tensors already scaled to [0, 1] (train.py:357 divides by 255).
    Returns loss5 = [pixel L1 (= F.l1_loss(pred, clean), train.py:365), tv1, tv2, cst, total].
    """

    def __init__(self, net: UNet, lr: float = 3e-4, n_epoch: int = 100, gamma: float = 0.5,
                 alpha_beta_gamma=(1.0, 0.5, 0.5), distributed: bool | None = None):
        self.net = net
        self.base_lr, self.n_epoch, self.gamma = lr, n_epoch, gamma
        self.weights = alpha_beta_gamma
        self.distributed = dp.require_group(distributed)
        if self.distributed:
            dp.broadcast_params(net.flat_params)
        self.opt = FlatAdam(net.flat_params, lr=lr)
        self.grad = torch.zeros_like(net.flat_params)
        self._bufs = {}

    def _buffers(self, N, C, H, W, device):
        key = (N, C, H, W, device)
        if key not in self._bufs:
            f = dict(dtype=torch.float32, device=device)
            self._bufs = {key: dict(
                inp=torch.empty((2 * N, C, H, W), **f),
                pred=torch.empty((2 * N, self.net.out_nc, H, W), **f),
                dpred=torch.empty((2 * N, self.net.out_nc, H, W), **f),
                loss5=torch.empty(5, **f),
                ws=self.net._workspace(2 * N, H, W, with_backward=True, fresh=True))}
        return self._bufs[key]

    def train_step(self, clean: torch.Tensor, noisy: torch.Tensor, epoch: int = 1) -> torch.Tensor:
        clean, noisy = clean.contiguous(), noisy.contiguous()
        if clean.shape != noisy.shape or clean.shape[1] != self.net.in_nc:
            raise ValueError("clean and noisy must share one [N, in_nc, H, W] shape")
        if self.net.in_nc != self.net.out_nc:
            raise ValueError("Structure_loss compares the output with the input: in_nc == out_nc")
        N, C, H, W = clean.shape
        b = self._buffers(N, C, H, W, clean.device)
        b["inp"][:N].copy_(noisy)
        b["inp"][N:].copy_(clean)
        self.net._run_forward(b["inp"], b["pred"], b["ws"])
        a, be, g = self.weights
        pred, pred2 = b["pred"][:N], b["pred"][N:]
        structure_loss_into(pred, pred2, clean, a, be, g, b["dpred"][:N], b["dpred"][N:], b["loss5"])
        self.net._run_backward(b["dpred"], self.grad, b["ws"], 2 * N, H, W)
        scale = dp.allreduce_grads(self.grad) if self.distributed else 1.0
        self.opt.lr = lr_at_epoch(epoch, self.base_lr, self.n_epoch, self.gamma)
        self.opt.step(self.grad, grad_scale=scale)
        return b["loss5"].clone()
