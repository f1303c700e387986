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
