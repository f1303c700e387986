"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference (lmh9507/image_denoising) hot path, used as the checker for
the HIP path.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import it; the product package `image_denoising_amd` never does (it has no CPU fallback).

  philox.py    counter-based Philox4x32-10 restated in numpy (bit-exact vs the HIP kernel)
  n2n_ref.py   train.py:134-190 sub-sampler (literal unfold/mask restatement + closed form),
               training_script.md:141-153 N2N loss, util.py:41-70 Structure_loss
  unet_ref.py  arch_unet.py:100-260 UNet forward as torch-CPU functional ops on the flat
               parameter buffer (autograd gives the backward), the N2N step with
               torch.optim.Adam (train.py:332)
  eval_ref.py  utils_eval.py:19-53 PSNR / SSIM restated with numpy

Pinned by tests/golden/*.npz, generated in the build container from the reference itself by
tests/golden/make_golden.py (see tests/test_oracle_golden.py).
"""
