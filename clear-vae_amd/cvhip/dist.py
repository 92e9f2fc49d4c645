"""Data-parallel plumbing of the fused CLEAR step (one process per GPU, torch.distributed over RCCL).

The reference trains on one device (code/src/trainer.py:435-493); its multi-GPU story is "wrap it in
torch DDP" (SURVEY.md section 8e).  The fused engine reproduces exactly those semantics without DDP:

  * every rank starts from rank 0's parameters (DDP broadcasts at construction): broadcast_flat;
  * every rank runs the full step on its own shard of the global batch (local-batch BatchNorm,
    contrastive and MI terms, as DDP around the reference would);
  * the flat gradient arena is SUM-all-reduced in buckets and the Adam kernel multiplies by
    1/world (cv_adam_step's grad_scale), i.e. gradients are averaged like DDP's.

Buckets follow the backward order: the decoder gradients are complete first, so their all-reduce is
launched (async, RCCL's own stream) while the encoder backward is still running; the encoder bucket
follows, and the optimizer waits for both.  Everything here is host logic over torch tensors, so it
runs on CPU tensors with the gloo backend in the tests.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist


def prepare_captured_collectives_env() -> None:
    """Call before creating an RCCL process group whose collectives a step graph will capture
    (CVHIP_GRAPH_COLLECTIVES=1).  A collective captured into the graph records its completion event inside
    the capture; with the process group's event cache on (its default) that event object is handed back to
    the cache and reused by a later eager collective, and the group's watchdog thread then fails querying it
    ("operation not permitted on an event last recorded in a capturing stream", seen intermittently in
    tests/test_gpu_graph_collectives.py).  Fresh events per collective remove the reuse."""
    if os.environ.get("CVHIP_GRAPH_COLLECTIVES", "0") == "1":
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


_CAPTURE_GROUP = None


def captured_collectives_group():
    """The process group a step graph captures its all-reduces on (CVHIP_GRAPH_COLLECTIVES=1).

    A dedicated RCCL group over every rank, constructed with its CUDA-event cache off
    (TORCH_NCCL_CUDA_EVENT_CACHE=0 while the group is built: ProcessGroupNCCL reads it in its constructor).
    With the cache on, a completion event recorded inside the capture goes back to the cache and is reused by a
    later eager collective, which the group's watchdog then fails to query ("operation not permitted on an event
    last recorded in a capturing stream", hipErrorCapturedEvent, an abort of the process).  The step's bucket
    collectives, eager first step included, run only on this group, so the default group's setting (whoever
    created it, whenever) cannot reach that abort.  Collective: every rank must call it, in the same order."""
    global _CAPTURE_GROUP
    if not (dist.is_available() and dist.is_initialized()):
        raise RuntimeError("captured collectives need an initialised torch.distributed process group")
    if dist.get_backend() != "nccl":
        raise RuntimeError("captured collectives need the nccl (RCCL) backend: a %r collective cannot be captured "
                           "into a HIP graph (unset CVHIP_GRAPH_COLLECTIVES)" % dist.get_backend())
    world_pg = dist.group.WORLD
    if _CAPTURE_GROUP is None or _CAPTURE_GROUP[0] is not world_pg:  # (none yet, or the default group was rebuilt)
        key = "TORCH_NCCL_CUDA_EVENT_CACHE"
        prev = os.environ.get(key)
        os.environ[key] = "0"
        try:
            _CAPTURE_GROUP = (world_pg, dist.new_group(backend="nccl"))
        finally:
            if prev is None:
                del os.environ[key]
            else:
                os.environ[key] = prev
    return _CAPTURE_GROUP[1]


def world() -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def rank() -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank()
    return 0


def shard_bounds(n_global: int, r: int, w: int) -> tuple:
    """Contiguous shard [lo, hi) of a global batch of n_global for rank r of w (sizes differ by <= 1)."""
    base, extra = divmod(n_global, w)
    lo = r * base + min(r, extra)
    return lo, lo + base + (1 if r < extra else 0)


def broadcast_flat(flat: torch.Tensor, src: int = 0, group=None) -> None:
    """Make every rank's flat parameter arena equal to rank src's (DDP's construction-time broadcast)."""
    if world() > 1:
        dist.broadcast(flat, src, group=group)


class GradBuckets:
    """Contiguous views of a flat gradient arena, all-reduced (SUM) in the order given.

    `bounds` are (lo, hi) element ranges in launch order; `launch(i)` starts bucket i's all-reduce
    asynchronously and `wait()` makes the current stream (or, for gloo, the host) wait for every
    launched bucket."""

    def __init__(self, flat: torch.Tensor, bounds: list, group=None, force: bool = False):
        """force: issue the collectives even in a world-1 process group (the one-GPU rehearsal of the RCCL path)."""
        self.flat = flat
        self.force = force
        self.bounds = list(bounds)
        self.views = [flat[lo:hi] for lo, hi in self.bounds]
        self.group = group
        self.pending = []
        covered = sorted(self.bounds)
        assert covered[0][0] == 0 and covered[-1][1] == flat.numel(), "buckets must cover the arena"
        for (a0, a1), (b0, b1) in zip(covered, covered[1:]):
            assert a1 == b0, "buckets must be contiguous and disjoint"

    def launch(self, i: int) -> None:
        if (world() > 1 or (self.force and dist.is_available() and dist.is_initialized())) and self.views[i].numel():
            self.pending.append(dist.all_reduce(self.views[i], op=dist.ReduceOp.SUM, group=self.group,
                                                async_op=True))

    def wait(self) -> None:
        for w in self.pending:
            w.wait()
        self.pending = []

    def reduce_all(self) -> None:
        for i in range(len(self.views)):
            self.launch(i)
        self.wait()


def average_in_place(flat: torch.Tensor, group=None) -> None:
    """Reference semantics of the engine's reduction: SUM all-reduce then scale by 1/world."""
    w = world()
    if w > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        flat.mul_(1.0 / w)
