"""The data-parallel PRODUCT path on the GPU: two ranks of N2NTrainer(distributed=True), each a
fresh process (tests/dp_worker.py) sharing the box's one MI355X over gloo, against the
single-process trainer on the concatenated batch (BASELINE configs[2]'s math: global-batch mean
gradient, replicas identical).  Rank 1 starts from perturbed weights, so the init broadcast is
under test; the loss, the all-reduced gradient and the post-Adam weights after two steps are
compared.  train.py:324-326 (nn.DataParallel) is the reference's version of this path."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("prec", ["fp32", "fp32_x6"])
def test_two_rank_n2n_trainer_equals_full_batch(tmp_path, prec):
    sys.path.insert(0, HERE)
    import dp_worker

    from image_denoising_amd import N2NTrainer

    out = str(tmp_path / "dp.npz")
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), out,
                                       prec], env=env, cwd=ROOT))
    try:
        codes = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert codes == [0, 0], codes
    r = np.load(out)
    assert np.array_equal(r["flat0"], r["flat1"])  # replicas identical after two updates
    # the single-process trainer on the whole batch
    net = dp_worker.build(prec, 0)
    tr = N2NTrainer(net, distributed=False)
    losses = dp_worker.run(tr, 0, 1).cpu().numpy()
    grad = tr.grad.cpu().numpy()
    flat = net.flat_params.detach().cpu().numpy()
    # step 1: same weights, the loss differs by summation order only; step 2 follows updates
    # that may differ by the sign flips below
    assert np.abs(r["losses"][0] - losses[0]).max() <= 1e-6 * np.abs(losses[0]).max()
    assert np.abs(r["losses"][1] - losses[1]).max() <= 1e-4 * np.abs(losses[1]).max()
    assert np.abs(r["grad"] - grad).max() <= 1e-4 * np.abs(grad).max()
    # Adam moves each weight by ~lr*sign(g) early on: a gradient within rounding of 0 may take
    # the other sign in the other summation order (as in test_n2n_step_vs_reference)
    d = np.abs(r["flat0"] - flat)
    assert (d > 1e-6).mean() < 2e-3, (d > 1e-6).mean()
    assert d.max() <= 2 * 2 * 3e-4 + 1e-6


def _two_rank_gloo(tmp_path, tag, prec, extra):
    out = str(tmp_path / f"{tag}.npz")
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1", **extra)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), out,
                                       prec], env=env, cwd=ROOT))
    try:
        codes = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert codes == [0, 0], codes
    return np.load(out)


def test_two_rank_bucketed_allreduce_equals_one_allreduce(tmp_path):
    """The overlapped gradient all-reduce (default: the decoder + head bucket all-reduced on a
    comm stream behind the library's tail-ready event, while the encoder's gradients are still
    computed; then the encoder bucket) against one all-reduce after the backward
    (DN_AR_OVERLAP=0), two ranks on the GPU over gloo: bit-identical losses, gradient and
    weights (the sums are elementwise, only their issue order moves)."""
    a = _two_rank_gloo(tmp_path, "bucketed", "fp32_x6", {"DN_AR_OVERLAP": "1"})
    b = _two_rank_gloo(tmp_path, "one", "fp32_x6", {"DN_AR_OVERLAP": "0"})
    for k in ("losses", "grad", "flat0", "flat1"):
        assert np.array_equal(a[k], b[k]), k


def test_one_rank_rccl_n2n_trainer_bit_exact(tmp_path):
    """The RCCL path itself (BASELINE configs[2]'s collective, train.py:324-326): a ONE-rank
    "nccl" process group on the box's GPU, started in a fresh process before any GPU call.
    N2NTrainer(distributed=True) broadcasts and all-reduces through RCCL every step; the
    one-rank sum is the identity and the scale 1, so two steps must equal a distributed=False
    run bit for bit."""
    out = str(tmp_path / "rccl.npz")
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), PYTHONUNBUFFERED="1")
    p = subprocess.run([sys.executable, os.path.join(HERE, "dp_worker.py"), out, "fp32_x6",
                        "nccl"], env=env, cwd=ROOT, timeout=240)
    assert p.returncode == 0
    r = np.load(out)
    assert str(r["backend"]) == "nccl"
    assert np.array_equal(r["losses"], r["losses_local"])
    assert np.array_equal(r["grad"], r["grad_local"])
    assert np.array_equal(r["flat"], r["flat_local"])


def test_single_stream_step_equals_two_stream_default(tmp_path):
    """DN_STEP_STREAMS=0 (the no-grad target pass on the main stream) and DN_BWD_STREAMS=0 (the
    weight gradients on the main stream) give the default two-stream step's results bit for bit
    (every kernel writes its own buffers; the streams only reorder independent launches).  The
    C++ side reads DN_BWD_STREAMS once per process, hence a fresh process per setting."""
    res = {}
    for tag, extra in (("two", {}), ("one", {"DN_STEP_STREAMS": "0", "DN_BWD_STREAMS": "0"})):
        out = str(tmp_path / f"{tag}.npz")
        env = dict(os.environ, PYTHONUNBUFFERED="1", **extra)
        for k in ("DN_STEP_STREAMS", "DN_BWD_STREAMS"):
            if k not in extra:
                env.pop(k, None)
        p = subprocess.run([sys.executable, os.path.join(HERE, "dp_worker.py"), out, "fp32_x6",
                            "local"], env=env, cwd=ROOT, timeout=240)
        assert p.returncode == 0, tag
        res[tag] = np.load(out)
    for k in ("losses", "grad", "flat"):
        assert np.array_equal(res["one"][k], res["two"][k]), k


@pytest.mark.parametrize("prec", ["fp32", "fp32_x6"])
def test_backward_with_padded_concat_strides(tmp_path, prec):
    """DN_C1S_ALIGN=32 pads every concat buffer's pixel stride (144 -> 160, 100 -> 128) in the
    backward plan too: the backward must take the channel count from the layer (ck), not from
    the stride, so outputs and every gradient equal the dense-stride plan's."""
    res = {}
    for tag, extra in (("dense", {}), ("pad32", {"DN_C1S_ALIGN": "32"})):
        out = str(tmp_path / f"{tag}.npz")
        env = dict(os.environ, PYTHONUNBUFFERED="1", **extra)
        if not extra:
            env.pop("DN_C1S_ALIGN", None)
        p = subprocess.run([sys.executable, os.path.join(HERE, "dp_worker.py"), out, prec, "grad"],
                           env=env, cwd=ROOT, timeout=240)
        assert p.returncode == 0, tag
        res[tag] = np.load(out)
    for k in ("y", "g", "dx"):
        a, b = res["dense"][k], res["pad32"][k]
        assert np.abs(a - b).max() <= 1e-5 * np.abs(a).max(), (k, np.abs(a - b).max())


def _worker_env_run(tmp_path, tag, extra, mode, prec="fp32_x6", shape="8,128,128"):
    """dp_worker.py on 8 x 128^2 (the 96-output convs at 128^2 take k_c3w6, the 48-channel
    encoder the pipelined kernels with the fused pool)"""
    out = str(tmp_path / f"{tag}.npz")
    env = dict(os.environ, PYTHONUNBUFFERED="1", DPW_SHAPE=shape, **extra)
    for k in ("DN_POOL_FUSE", "DN_X6_W6", "DN_X6_RING3", "DN_W6_MIN_TILES"):
        if k not in extra:
            env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(HERE, "dp_worker.py"), out, prec, mode],
                       env=env, cwd=ROOT, timeout=240)
    assert p.returncode == 0, tag
    return np.load(out)


def test_fused_pool_step_equals_separate_pool(tmp_path):
    """The encoder's 2x2 max-pools fused into the x6 convs' epilogue (default) give the N2N step
    of separate k_pool_fwd launches (DN_POOL_FUSE=0) bit for bit: the same activated values,
    the same window order."""
    fused = _worker_env_run(tmp_path, "fused", {}, "local")
    sep = _worker_env_run(tmp_path, "sep", {"DN_POOL_FUSE": "0"}, "local")
    for k in ("losses", "grad", "flat"):
        assert np.array_equal(fused[k], sep[k]), k


def test_small_grid_ring_step_equals_single_stage_prefetch(tmp_path):
    """Below one round of 16 x 16 tiles (here every level under 64^2 of the 8 x 128^2 step) the
    3x3 convs run on k_c3x6h with a 3-slot weight ring (default) instead of k_c3x6
    (DN_X6_RING3=0): the same products in the same order, so the N2N step is bit-identical."""
    ring = _worker_env_run(tmp_path, "ring3", {}, "local")
    old = _worker_env_run(tmp_path, "noring", {"DN_X6_RING3": "0"}, "local")
    for k in ("losses", "grad", "flat"):
        assert np.array_equal(ring[k], old[k]), k


def test_winograd_step_matches_direct_kernels(tmp_path):
    """The 96-output 3x3 convs on the 1-D Winograd kernel k_c3w6 (default) against the direct
    bf16x6 kernels (DN_X6_W6=0): the same arithmetic class (fp32-accurate dot products; the
    transform adds one rounding of v and u), so outputs and every gradient agree to fp32
    rounding.  Tolerance: 2e-5 of the max magnitude for the output and the parameter gradients
    (LeakyReLU's slope switch at 0 can move a gradient element by rounding, as between any two
    fp32 implementations).  dL/dx of this random-init net is ~1e-16, i.e. a sum of much larger
    terms that cancel to rounding level, so only its scale is compared (5e-2)."""
    w6 = _worker_env_run(tmp_path, "w6", {}, "grad")
    d = _worker_env_run(tmp_path, "direct", {"DN_X6_W6": "0"}, "grad")
    for k, tol in (("y", 2e-5), ("g", 2e-5), ("dx", 5e-2)):
        a, b = w6[k], d[k]
        assert np.abs(a - b).max() <= tol * np.abs(a).max(), (k, np.abs(a - b).max())


def test_improved_unet_winograd_blocks_match_direct_kernels(tmp_path):
    """ImprovedUNet's 96 / 192 / 384-channel 3x3 forwards and data gradients on k_c3w6 in
    96-channel output blocks (blockIdx.z: the per-block image stride wp_z, the channel offset of
    the epilogue) against the direct bf16x6 kernels (DN_X6_W6=0).  DN_W6_MIN_TILES=1 routes every
    96-block launch to the Winograd kernel at this test size (the default takes it from one
    round of 512 tiles, i.e. at the bench's 64 x 256^2).  Same arithmetic class, so the output
    agrees to 2e-5 of its max magnitude, as the UNet test above.  The parameter gradients go
    through ImprovedUNet's GroupNorm backward, which amplifies fp32 rounding differences
    (test_gpu_iunet compares them per tensor at 1e-3 against the oracle); measured here 2.0e-5 of
    the max gradient, bound 1e-4 (an indexing or block-offset error is O(1))."""
    w6 = _worker_env_run(tmp_path, "iw6", {"DN_W6_MIN_TILES": "1"}, "igrad", shape="2,64,64")
    d = _worker_env_run(tmp_path, "idirect", {"DN_X6_W6": "0"}, "igrad", shape="2,64,64")
    a, b = w6["y"], d["y"]
    assert np.abs(a - b).max() <= 2e-5 * np.abs(a).max(), np.abs(a - b).max()
    ga = np.concatenate([w6[f"g{i}"] for i in range(len(w6["names"]))])
    gb = np.concatenate([d[f"g{i}"] for i in range(len(d["names"]))])
    assert np.abs(ga - gb).max() <= 1e-4 * np.abs(ga).max(), np.abs(ga - gb).max()
