"""Data parallelism for the N2N step: one process per GPU, RCCL over xGMI.

Replaces train.py:324-326 (single-process nn.DataParallel: per-forward parameter broadcast,
scatter, threaded replicas, gather, grad reduce-add onto GPU 0) with the one exchange the path
really has: ONE all-reduce(sum) of the flat fp32 gradient buffer per step (1,256,689 floats =
5.03 MB for in=out=1), scaled by 1/world inside the fused Adam kernel.  Parameters are
broadcast once at start-up; replicas then stay identical because every rank applies the same
deterministic Adam update to the same reduced gradient.

Sharding: the global batch of B patches is split contiguously, rank r owning patches
[r*b, (r+1)*b) with b = B/world.  The counter-based random streams (noise, neighbour masks)
are indexed by GLOBAL element / cell numbers via the bases below, so a patch sees the same
noise and mask pair whatever the world size.  The loss is a mean over the local batch, so the
average of the ranks' gradients equals the gradient of the global-batch mean (equal shards).

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on the GPU box, "gloo" for
the CPU tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


# The step's own streams, one of each kind per device: "side" (the N2N no-grad pass beside the
# gradient pass) and "comm" (the early gradient bucket's all-reduce).  HIP binds a stream to one
# of GPU_MAX_HW_QUEUES (default 4) hardware queues at its first submission and shares queues
# after that; streams sharing a queue run one after the other.  In a one-rank RCCL run the no-grad
# pass shared the main stream's queue (RCCL's streams had taken the free ones first): 19.34-19.45
# against 18.97 ms/step for the plain bench; with prepare_streams() (the step's streams touched
# before the process group exists) 19.08-19.18 against 18.92-19.01 (profiles/r6_dp1_streams.log).
# Raising GPU_MAX_HW_QUEUES instead made every launch slower (8: +0.8, 16: +1.3 ms/step under
# torchrun, profiles/r6_hwq.log).
_STEP_STREAMS: dict = {}


def step_stream(kind: str, device) -> torch.cuda.Stream:
    """the cached stream `kind` ("side" / "comm") of `device`"""
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:  # "cuda" and "cuda:<current>" share one
        device = torch.device("cuda", torch.cuda.current_device())
    key = (kind, device)
    st = _STEP_STREAMS.get(key)
    if st is None:
        st = _STEP_STREAMS[key] = torch.cuda.Stream(device=device)
    return st


def prepare_streams(device) -> None:
    """First submissions on the streams whose work runs concurrently in the step -- the no-grad
    pass's, then the library's weight-gradient and reduction streams -- so that with the main
    stream they hold the four hardware queues before RCCL creates its streams.  The comm stream
    comes last: it (like RCCL's streams) only carries work enqueued after the whole backward, so
    sharing a queue costs it nothing but overlap, while a shared queue between two of the compute
    streams serialises them."""
    from . import _lib

    device = torch.device(device)
    with torch.cuda.stream(step_stream("side", device)):
        torch.zeros(1, device=device)
    _lib.call("dn_prepare_streams", torch.cuda.current_stream(device).cuda_stream)
    with torch.cuda.stream(step_stream("comm", device)):
        torch.zeros(1, device=device)


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def is_distributed() -> bool:
    """a process group with more than one rank: what a trainer built with distributed=None
    (auto) takes as "run data-parallel".  A trainer built with distributed=True runs its
    collectives on any initialised group, world 1 included (a one-rank RCCL group exercises the
    same broadcast / all-reduce calls as eight)."""
    return is_initialized() and dist.get_world_size() > 1


def require_group(distributed: bool | None) -> bool:
    """resolve a trainer's `distributed` argument: None -> is_distributed(); True -> an
    initialised process group is required (ValueError otherwise)"""
    if distributed is None:
        return is_distributed()
    if distributed and not is_initialized():
        raise ValueError("distributed=True needs an initialised torch.distributed process group "
                         "(image_denoising_amd.dist.init_from_env)")
    return bool(distributed)


def launched_by_torchrun() -> bool:
    """torchrun / torch.distributed.run sets TORCHELASTIC_RUN_ID for every rank it starts"""
    return "TORCHELASTIC_RUN_ID" in os.environ


def world_and_rank() -> tuple[int, int]:
    if is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def init_from_env(backend: str = "nccl", force: bool = False) -> tuple[int, int, int]:
    """torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT) -> process group.
    Returns (world, rank, local_rank).  The group is created when world > 1, when torchrun
    started this process (any world size: `torchrun --nproc-per-node 1` runs a one-rank RCCL
    group) or when `force` is set; a plain single process stays non-distributed."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    want = world > 1 or force or launched_by_torchrun()
    if want and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            prepare_streams(torch.device("cuda", local))
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def shard_bases(rank: int, local_batch: int, channels: int, height: int, width: int):
    """(elem_base, cell_base): global index of this rank's first noise element and first 2x2
    sub-sampler cell."""
    elem_base = rank * local_batch * channels * height * width
    cell_base = rank * local_batch * (height // 2) * (width // 2)
    return elem_base, cell_base


def broadcast_params(flat: torch.Tensor, src: int = 0) -> None:
    """rank src's parameters to every rank (any initialised group, world 1 included)"""
    if is_initialized():
        dist.broadcast(flat, src=src)


def allreduce_grads(flat_grad: torch.Tensor) -> float:
    """Sum the flat gradient over ranks in place (any initialised group, world 1 included);
    returns the scale (1/world) the optimizer applies, so the update uses the global-batch mean
    gradient."""
    if not is_initialized():
        return 1.0
    dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM)
    return 1.0 / dist.get_world_size()


def allreduce_grads_split(flat_grad: torch.Tensor, tail_begin: int, run_backward,
                          comm_stream=None) -> float:
    """The gradient all-reduce overlapped with the backward (two buckets; train.py:324-326
    reduces during its backward too).  run_backward(event) enqueues the backward and has the
    library record `event` once flat_grad[tail_begin:] (the decoder and the head, finished
    first) is final; that bucket's all-reduce is enqueued on `comm_stream` behind the event,
    so it runs while the encoder's gradients are still being computed, and the encoder bucket
    flat_grad[:tail_begin] follows on the current stream behind the whole backward.  The
    current stream then waits for both.  At world 2 every element is one a + b, so the result
    equals allreduce_grads' bit for bit; from 3 ranks on, a ring all-reduce's per-element
    summation order follows the chunk the element falls in, and moving the chunk boundaries
    (two buckets) may change the last bits: equal up to fp32 summation order.  CPU tensors (the gloo tests): run_backward(None), then the
    same two buckets in the same order.  Returns 1/world like allreduce_grads."""
    if not is_initialized():
        run_backward(None)
        return 1.0
    tail, head = flat_grad[tail_begin:], flat_grad[:tail_begin]
    if flat_grad.device.type != "cuda" or comm_stream is None:
        run_backward(None)
        dist.all_reduce(tail, op=dist.ReduceOp.SUM)
        dist.all_reduce(head, op=dist.ReduceOp.SUM)
        return 1.0 / dist.get_world_size()
    ev = torch.cuda.Event()
    ev.record()  # materialise the event; the library re-records it mid-backward
    run_backward(ev)
    comm_stream.wait_event(ev)
    with torch.cuda.stream(comm_stream):
        w_tail = dist.all_reduce(tail, op=dist.ReduceOp.SUM, async_op=True)
    w_head = dist.all_reduce(head, op=dist.ReduceOp.SUM, async_op=True)
    w_tail.wait()
    w_head.wait()
    return 1.0 / dist.get_world_size()


def allreduce_mean_(t: torch.Tensor) -> torch.Tensor:
    """mean of a (small) tensor over ranks, e.g. the logged loss (no host sync involved)"""
    if is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t /= dist.get_world_size()
    return t
