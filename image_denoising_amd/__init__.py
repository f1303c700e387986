"""image_denoising_amd — MI355X-native Neighbor2Neighbor U-Net training path.

Drop-in for the hot path of lmh9507/image_denoising (arch_unet.UNet, train.py's N2N
sub-sampler, the N2N / Structure losses, Adam) computed by hand-written gfx950 HIP kernels
behind the C-ABI of libdenoise_hip.so (include/denoise_hip.h).
"""
from .adapter import DenoiserWithAdapter, OutputAdapter  # noqa: F401
from .arch_unet import UNet, reference_init  # noqa: F401
from .finetune import FinetuneTrainer  # noqa: F401
from .improved_unet import ImprovedUNet  # noqa: F401
from .n2n import (AugmentNoise, generate_mask_pair, generate_subimages,  # noqa: F401
                  n2n_loss, n2n_subsample)
from .optim import FlatAdam, lr_at_epoch  # noqa: F401
from .trainer import N2NTrainer, StructureTrainer  # noqa: F401
from .util import Structure_loss  # noqa: F401

__version__ = "0.1.0"
