"""ctypes binding of libdenoise_hip.so (include/denoise_hip.h).

The product path has no fallback: if the HIP library is missing or fails to load, importing
anything that computes raises.  Tensors cross the boundary as raw device pointers; the HIP
stream is torch's current stream on the tensor's device.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int64, c_size_t, c_uint8, c_uint64, c_void_p

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DN_LIB_PATH", os.path.join(_HERE, "libdenoise_hip.so"))


ABI_VERSION = 5  # include/denoise_hip.h DN_ABI_VERSION


class DnOpRecord(ctypes.Structure):  # include/denoise_hip.h dn_op_record
    _fields_ = [("op", ctypes.c_char * 24), ("kernel", ctypes.c_char * 48), ("K", c_int),
                ("NOUT", c_int), ("H", c_int), ("W", c_int), ("N", c_int),
                ("flops", ctypes.c_double), ("ms", ctypes.c_double)]


class DnCfg(ctypes.Structure):
    _fields_ = [("in_nc", c_int), ("out_nc", c_int), ("n_feature", c_int)]


_F = c_void_p  # float*  (device)
_U8 = c_void_p  # uint8_t* (device)

# name -> (restype, argtypes)
SIGNATURES = {
    "dn_version": (c_char_p, []),
    "dn_abi_version": (c_int, []),
    "dn_profile_ops": (c_int, [c_int]),
    "dn_prepare_streams": (c_int, [c_void_p]),
    "dn_profile_ops_read": (c_int, [c_void_p, c_int, POINTER(c_int)]),
    "dn_last_error": (c_int, [c_char_p, c_size_t]),
    "dn_unet_param_count": (c_int, [POINTER(DnCfg), POINTER(c_size_t)]),
    "dn_unet_param_info": (c_int, [POINTER(DnCfg), c_int, POINTER(c_size_t), POINTER(c_size_t),
                                   POINTER(c_size_t)]),
    "dn_unet_workspace_size": (c_int, [POINTER(DnCfg), c_int, c_int, c_int, c_int,
                                       POINTER(c_size_t)]),
    "dn_unet_forward": (c_int, [POINTER(DnCfg), _F, _F, _F, c_int, c_int, c_int, c_void_p,
                                c_size_t, c_void_p]),
    "dn_unet_backward": (c_int, [POINTER(DnCfg), _F, _F, _F, _F, c_int, c_int, c_int, c_void_p,
                                 c_size_t, c_void_p]),
    "dn_unet_forward_bf16": (c_int, [POINTER(DnCfg), _F, _F, _F, c_int, c_int, c_int, c_void_p,
                                     c_size_t, c_void_p]),
    "dn_unet_forward_n2n": (c_int, [POINTER(DnCfg), _F, _F, _F, _U8, c_int, c_int, c_int,
                                    c_void_p, c_size_t, c_int, c_void_p]),
    "dn_unet_forward_prec": (c_int, [POINTER(DnCfg), _F, _F, _F, c_int, c_int, c_int, c_void_p,
                                     c_size_t, c_int, c_void_p]),
    "dn_unet_pack_weights": (c_int, [POINTER(DnCfg), _F, c_int, c_int, c_int, c_void_p, c_size_t,
                                     c_int, c_void_p]),
    "dn_unet_forward_prepacked": (c_int, [POINTER(DnCfg), _F, _F, _F, c_int, c_int, c_int,
                                          c_void_p, c_size_t, c_int, c_void_p]),
    "dn_unet_backward_prec": (c_int, [POINTER(DnCfg), _F, _F, _F, _F, c_int, c_int, c_int,
                                      c_void_p, c_size_t, c_int, c_void_p]),
    "dn_unet_backward_split": (c_int, [POINTER(DnCfg), _F, _F, _F, _F, c_int, c_int, c_int,
                                       c_void_p, c_size_t, c_int, c_void_p, c_void_p,
                                       POINTER(c_int64)]),
    "dn_unet_debug_buffers": (c_int, [POINTER(DnCfg), c_int, c_int, c_int, c_int,
                                      POINTER(c_int64), c_int, POINTER(c_int)]),
    "dn_n2n_subsample": (c_int, [_F, c_int, c_int, c_int, c_int, _U8, c_uint64, c_uint64, c_uint64,
                                 _F, _F, _U8, c_void_p]),
    "dn_n2n_masks": (c_int, [_U8, c_int64, _U8, _U8, c_void_p]),
    "dn_n2n_subimage_from_mask": (c_int, [_F, c_int, c_int, c_int, c_int, _U8, _F, c_void_p]),
    "dn_add_gauss_noise": (c_int, [_F, c_int, c_int64, c_float, _F, c_uint64, c_uint64, c_uint64,
                                   _F, c_void_p]),
    "dn_add_poisson_noise": (c_int, [_F, c_int, c_int64, c_float, _F, c_uint64, c_uint64, c_uint64,
                                   _F, c_void_p]),
    "dn_loss_partials_size": (c_size_t, []),
    "dn_n2n_loss": (c_int, [_F, _F, _F, _U8, c_int, c_int, c_int, c_int, c_float, _F, _F, c_void_p,
                            c_void_p]),
    "dn_structure_loss": (c_int, [_F, _F, _F, c_int, c_int, c_int, c_int, c_float, c_float,
                                  c_float, _F, _F, _F, c_void_p, c_void_p]),
    "dn_adam_step": (c_int, [_F, _F, _F, _F, c_int64, c_float, c_float, c_float, c_float, c_int64,
                             c_float, c_void_p]),
    "dn_conv2d_pack_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "dn_deconv2x2_pack_size": (c_size_t, [c_int, c_int, c_int]),
    "dn_conv2d_forward": (c_int, [_F, c_int, c_int, c_int, c_int, c_int, _F, _F, c_int, c_int,
                                  c_int, _F, c_int, c_void_p, c_size_t, c_void_p]),
    "dn_conv2d_bf16_pack_size": (c_size_t, [c_int, c_int]),
    "dn_conv2d_forward_bf16": (c_int, [_F, c_int, c_int, c_int, c_int, c_int, _F, _F, c_int, c_int,
                                       _F, c_int, c_void_p, c_size_t, c_void_p]),
    "dn_conv2d_x6_pack_size": (c_size_t, [c_int, c_int, c_int]),
    "dn_conv2d_forward_x6": (c_int, [_F, c_int, c_int, c_int, c_int, c_int, _F, _F, c_int, c_int,
                                     _F, c_int, c_void_p, c_size_t, c_void_p]),
    "dn_conv2d_backward_data_x6": (c_int, [_F, c_int, c_int, c_int, c_int, _F, c_int, _F, c_int,
                                           c_int, _F, c_int, c_void_p, c_size_t, c_void_p]),
    "dn_conv2d_backward_data": (c_int, [_F, c_int, c_int, c_int, c_int, _F, c_int, c_int, _F,
                                        c_int, c_int, _F, c_int, c_void_p, c_size_t, c_void_p]),
    "dn_conv2d_wgrad_slab_size": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "dn_conv2d_backward_weight": (c_int, [_F, _F, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                          _F, c_void_p, c_void_p]),
    "dn_conv2d_backward_weight_x6": (c_int, [_F, _F, c_int, c_int, c_int, c_int, c_int, c_int,
                                             _F, c_void_p, c_void_p]),
    "dn_deconv2x2_forward": (c_int, [_F, c_int, c_int, c_int, c_int, _F, _F, c_int, _F, c_int,
                                     c_int, c_void_p, c_size_t, c_void_p]),
    "dn_deconv2x2_x6_pack_size": (c_size_t, []),
    "dn_deconv2x2_forward_x6": (c_int, [_F, c_int, c_int, c_int, _F, _F, _F, c_int, c_int, c_void_p,
                                        c_size_t, c_void_p]),
    "dn_deconv2x2_backward_data_x6": (c_int, [_F, c_int, c_int, c_int, c_int, _F, _F, _F, c_void_p,
                                              c_size_t, c_void_p]),
    "dn_deconv2x2_backward_data": (c_int, [_F, c_int, c_int, c_int, c_int, c_int, _F, c_int, _F,
                                           _F, c_void_p, c_size_t, c_void_p]),
    "dn_deconv2x2_wgrad_slab_size": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "dn_deconv2x2_backward_weight": (c_int, [_F, c_int, _F, c_int, c_int, c_int, c_int, c_int, _F,
                                             c_void_p, c_void_p]),
    "dn_maxpool2x2_forward": (c_int, [_F, c_int, c_int, c_int, c_int, _F, c_int, c_int, c_void_p]),
    "dn_maxpool2x2_backward": (c_int, [_F, c_int, c_int, c_int, c_int, _F, c_int, c_int, c_int, _F,
                                       c_void_p]),
    "dn_accumulate": (c_int, [_F, _F, c_int64, c_void_p]),
    "dn_eval_partials_size": (c_size_t, []),
    "dn_u8_to_unit": (c_int, [_U8, c_int64, _F, c_void_p]),
    "dn_tile_count": (c_int, [c_int, c_int, c_int]),
    "dn_tile_extract": (c_int, [_U8, c_int, c_int, c_int, c_int, c_int, _F, c_void_p]),
    "dn_tile_blend": (c_int, [_F, c_int, c_int, c_int, c_int, c_int, _F, _F, _U8, c_void_p]),
    "dn_quantize_u8": (c_int, [_F, c_int64, c_int, _U8, c_void_p]),
    "dn_psnr_u8": (c_int, [_U8, _U8, c_int64, c_void_p, c_void_p, c_void_p]),
    "dn_ssim_u8": (c_int, [_U8, _U8, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "dn_l1_mean_batched": (c_int, [_F, _F, c_int64, c_int64, c_void_p, c_void_p]),
    "dn_l1_mean": (c_int, [_F, _F, c_int64, c_void_p, c_void_p, c_void_p]),
    "dn_iunet_param_count": (c_int, [POINTER(DnCfg), POINTER(c_size_t)]),
    "dn_iunet_workspace_size": (c_int, [POINTER(DnCfg), c_int, c_int, c_int, c_int,
                                        POINTER(c_size_t)]),
    "dn_iunet_forward": (c_int, [POINTER(DnCfg), _F, _F, _F, c_int, c_int, c_int, c_void_p,
                                 c_size_t, c_void_p]),
    "dn_iunet_backward": (c_int, [POINTER(DnCfg), _F, _F, _F, c_int, c_int, c_int, c_void_p,
                                  c_size_t, c_void_p]),
    "dn_iunet_forward_prec": (c_int, [POINTER(DnCfg), _F, _F, _F, c_int, c_int, c_int, c_void_p,
                                      c_size_t, c_int, c_void_p]),
    "dn_iunet_backward_prec": (c_int, [POINTER(DnCfg), _F, _F, _F, c_int, c_int, c_int, c_void_p,
                                       c_size_t, c_int, c_void_p]),
    "dn_iunet_debug_buffers": (c_int, [POINTER(DnCfg), c_int, c_int, c_int, c_int,
                                       POINTER(c_int64), c_int, POINTER(c_int)]),
    "dn_adapter_param_count": (c_int, [c_int, c_int, POINTER(c_size_t)]),
    "dn_adapter_forward": (c_int, [_F, _F, _F, _F, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "dn_adapter_slab_size": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "dn_adapter_backward": (c_int, [_F, _F, _F, _F, _F, c_int, c_int, c_int, c_int, c_int,
                                    c_void_p, c_size_t, c_void_p]),
    "dn_finetune_loss": (c_int, [_F, _F, c_int, c_int, c_int, c_int, c_float, _F, _F, c_void_p,
                                 c_void_p]),
}

_lib = None


def lib() -> ctypes.CDLL:
    """The loaded library (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libdenoise_hip.so not found at {LIB_PATH}; build it with "
                "`python -m image_denoising_amd._build` (hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        L.dn_abi_version.restype = c_int
        if L.dn_abi_version() != ABI_VERSION:  # the argument lists below are revision 5's
            raise RuntimeError(f"{LIB_PATH}: ABI revision {L.dn_abi_version()}, the binding "
                               f"expects {ABI_VERSION} (include/denoise_hip.h DN_ABI_VERSION)")
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    buf = ctypes.create_string_buffer(2048)
    lib().dn_last_error(buf, 2048)
    return buf.value.decode(errors="replace")


class DenoiseHipError(RuntimeError):
    pass


def check(status: int, what: str) -> None:
    if status != 0:
        raise DenoiseHipError(f"{what} failed (status {status}): {last_error()}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def ptr(t: torch.Tensor | None):
    """device pointer of a contiguous tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return t.data_ptr()


def stream_of(t: torch.Tensor):
    if t.device.type != "cuda":
        raise ValueError(f"expected a GPU tensor, got device {t.device}")
    return torch.cuda.current_stream(t.device).cuda_stream


def scratch(nbytes: int, device) -> torch.Tensor:
    """caller-owned device scratch (the library never allocates)"""
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def cfg(in_nc: int, out_nc: int, n_feature: int) -> DnCfg:
    return DnCfg(in_nc, out_nc, n_feature)


def profile_ops(enable: bool) -> None:
    """dn_profile_ops: record every launch of the executors (single-stream) until disabled"""
    check(lib().dn_profile_ops(int(bool(enable))), "dn_profile_ops")


def profile_ops_take(cap: int = 8192) -> list[dict]:
    """waits for and returns the launch records since profile_ops(True), dropping them"""
    buf = (DnOpRecord * cap)()
    n = c_int(0)
    check(lib().dn_profile_ops_read(buf, cap, ctypes.byref(n)), "dn_profile_ops_read")
    if n.value > cap:
        raise RuntimeError(f"{n.value} launch records, only {cap} read")
    return [dict(op=r.op.decode(), kernel=r.kernel.decode(), K=r.K, NOUT=r.NOUT, H=r.H, W=r.W,
                 N=r.N, flops=r.flops, ms=r.ms) for r in buf[:n.value]]
