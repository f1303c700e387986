"""Stage timeline of k_c3x6p from the s_memtime stamps of a DN_X6_STAMPS=1 build:
    DN_BUILD_TAG=stamps DN_EXTRA_CXXFLAGS=-DDN_X6_STAMPS=1 python -m image_denoising_amd._build
    DN_LIB_PATH=image_denoising_amd/libdenoise_hip_stamps.so python tools/x6_stamps.py [K NOUT H]
Prints, in shader cycles (mean over the first 64 tiles of image 0, waves 0 and 4): the prologue,
per stage the compute span (opening barrier -> last MFMA issued), the tail (-> closing barrier
reached: x split, weight DMA issue, vmcnt wait) and the barrier wait, and the epilogue."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_denoising_amd import _lib  # noqa: E402

K, NO, H = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (96, 96, 256)))
N = int(os.environ.get("N", "64"))
dev = torch.device("cuda", 0)
x = torch.randn(N, H, H, K, device=dev)
w = torch.randn(NO, K, 3, 3, device=dev) * 0.05
b = torch.zeros(NO, device=dev)
y = torch.empty(N, H, H, NO, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
pk = _lib.scratch(_lib.lib().dn_conv2d_x6_pack_size(K, NO, 0), dev)
L = _lib.lib()
fn = L.dn_debug_x6_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
for _ in range(int(os.environ.get("REPS", "3"))):
    _lib.call("dn_conv2d_forward_x6", x.data_ptr(), K, N, H, H, NO, w.data_ptr(), b.data_ptr(), NO, 1,
              y.data_ptr(), NO, pk.data_ptr(), pk.numel(), s)
torch.cuda.synchronize()
SLOTS = 128
buf = np.zeros(64 * 2 * SLOTS, dtype=np.uint64)
assert fn(buf.ctypes.data, buf.size) == 0
st = buf.reshape(64, 2, SLOTS).astype(np.int64)
nst = 9 * ((K + 31) // 32)
A = st[:, :, 1:1 + 3 * nst:3]
C = st[:, :, 2:2 + 3 * nst:3]
E = st[:, :, 3:3 + 3 * nst:3]
loop_end = st[:, :, 1 + 3 * nst]
epi_end = st[:, :, 2 + 3 * nst]
epi_issued = st[:, :, 3 + 3 * nst]
start = st[:, :, 0]
nxt = np.concatenate([A[:, :, 1:], loop_end[:, :, None]], axis=2)
comp, tail, barw = C - A, E - C, nxt - E
tile = epi_end - start
print(f"k_c3x6p {K}->{NO} @{N}x{H}x{H}: {nst} stages, shader cycles (mean over 64 tiles x waves 0/4)")
print(f"  tile {tile.mean():9.0f}   prologue {(A[:, :, 0] - start).mean():7.0f}   "
      f"main loop {(loop_end - A[:, :, 0]).mean():9.0f}   epilogue {(epi_end - loop_end).mean():7.0f} "
      f"(issued {(epi_issued - loop_end).mean():7.0f}, store drain {(epi_end - epi_issued).mean():6.0f})")
print(f"  per stage: compute {comp.mean():6.0f}  tail {tail.mean():5.0f}  barrier {barw.mean():5.0f}"
      f"  (stage {(nxt - A).mean():6.0f}; MFMA floor 2 waves x 72 x 16 = 2304)")
for t in range(9):
    sl = slice(t, nst, 9)
    print(f"  tap {t}: compute {comp[:, :, sl].mean():6.0f}  tail {tail[:, :, sl].mean():5.0f}  "
          f"barrier {barw[:, :, sl].mean():5.0f}")
print("  wave 0 vs 4 compute:", comp[:, 0].mean().round(), comp[:, 1].mean().round())
