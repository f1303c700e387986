"""Builds libdenoise_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

    python -m image_denoising_amd._build        # incremental
    python -m image_denoising_amd._build --force
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
# DN_BUILD_TAG=t + DN_EXTRA_CXXFLAGS: a variant library libdenoise_hip_t.so (objects in _objs_t)
# for same-box A/B runs (DN_LIB_PATH selects it at load time); the default build has no tag
TAG = os.environ.get("DN_BUILD_TAG", "")
BUILD = os.path.join(PKG, "_objs" + (f"_{TAG}" if TAG else ""))
LIB = os.path.join(PKG, "libdenoise_hip" + (f"_{TAG}" if TAG else "") + ".so")
SOURCES = ["conv.hip", "conv_bf16.hip", "conv_x6.hip", "conv_w6.hip", "wgrad_x6p.hip", "elementwise.hip", "first_layer.hip", "eval.hip", "adapter.hip", "iunet_ops.hip", "unet.cpp",
           "iunet.cpp", "capi.cpp", "profile.cpp"]
HEADERS = ["dn_internal.h", "conv_epi.h", "x6_core.h", "philox.h", "unet.h", "iunet.h", "iunet_ops.h"]
ARCH = os.environ.get("DN_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
            "-Wno-unused-function", "-Wno-unused-variable",
            *os.environ.get("DN_EXTRA_CXXFLAGS", "").split()]
# the bf16x6 kernels keep their fp32 adds scalar: the SLP vectorizer would pair them into
# v_pk_add_f32, which costs more issue cycles beside MFMAs than the two adds (x6_core.h)
# conv_w6.hip: LLVM's max-memory-clause scheduling strategy, 19.10 -> 19.05 ms/step over six
# same-box pairs (profiles/r5_w6_sched_ab.log); for every file it slowed the weight gradients
FILE_FLAGS = {"conv_x6.hip": ["-fno-slp-vectorize"],
              "conv_w6.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
              "wgrad_x6p.hip": ["-fno-slp-vectorize"]}


def source_hash() -> str:
    """sha256 (first 16 hex digits) over the effective compile flags (CXXFLAGS including
    DN_EXTRA_CXXFLAGS, and every per-file flag set) and the library's sources, headers and C-ABI
    header, in a fixed order.  Compiled into dn_version() so a test can tie a loaded .so to the
    tree; a flag-only change rebuilds every object (the stamp in build() differs)."""
    h = hashlib.sha256()
    h.update(" ".join([HIPCC, *CXXFLAGS]).encode() + b"\0")
    for f in sorted(FILE_FLAGS):
        h.update(f.encode() + b":" + " ".join(FILE_FLAGS[f]).encode() + b"\0")
    paths = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    paths.append(os.path.join(ROOT, "include", "denoise_hip.h"))
    for p in paths:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _newest_header() -> float:
    paths = [os.path.join(CSRC, h) for h in HEADERS]
    paths.append(os.path.join(ROOT, "include", "denoise_hip.h"))
    return max(os.path.getmtime(p) for p in paths)


def _compile(src: str, force: bool, src_hash: str) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(BUILD, src + ".o")
    if not force and os.path.exists(o):
        if os.path.getmtime(o) >= max(os.path.getmtime(s), _newest_header()):
            return o
    cmd = [HIPCC, *CXXFLAGS, *FILE_FLAGS.get(src, []), "-x", "hip", "-c", s, "-o", o, f"-I{CSRC}",
           f"-I{os.path.join(ROOT, 'include')}", f'-DDN_SRC_HASH="{src_hash}"']
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip():
        sys.stderr.write(r.stderr)
    return o


def build(force: bool = False, jobs: int = 4) -> str:
    os.makedirs(BUILD, exist_ok=True)
    # the mtime checks below are only a shortcut: a tree whose sources hash differently from
    # the last build (a checkout, a copied tree) rebuilds everything
    src_hash = source_hash()
    stamp = os.path.join(BUILD, "src_hash")
    if not os.path.exists(stamp) or open(stamp).read().strip() != src_hash:
        force = True
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, src_hash), SOURCES))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(map(os.path.getmtime, objs)):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(src_hash)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
