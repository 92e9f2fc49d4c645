"""CVHIP_GRAPH_COLLECTIVES=1 (cvhip/engine.py, cvhip/dist.py): the captured-collectives abort (the RCCL watchdog's
hipErrorCapturedEvent on a cached event recorded inside a capture, round 5) cannot be reached through the caller's
setup.  The step's bucket collectives run on a dedicated group that cvhip.dist builds with the event cache off, and
a backend that cannot be captured is refused before anything is captured.  CPU-only: a world-1 gloo group, with
torch.distributed's group constructor observed (the RCCL form runs in tests/test_gpu_graph_collectives.py).
Reference step: /root/reference/code/src/trainer.py:861-888."""

import os
import socket

import pytest
import torch.distributed as dist

from cvhip import dist as cvdist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def gloo_world1():
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        yield
    finally:
        dist.destroy_process_group()
        cvdist._CAPTURE_GROUP = None


def test_refuses_uncapturable_backend(gloo_world1):
    with pytest.raises(RuntimeError, match="nccl"):
        cvdist.captured_collectives_group()


def test_refuses_without_process_group():
    assert not dist.is_initialized()
    with pytest.raises(RuntimeError, match="initialised"):
        cvdist.captured_collectives_group()


@pytest.mark.parametrize("caller_env", [None, "1"])
def test_dedicated_group_built_with_event_cache_off(gloo_world1, monkeypatch, caller_env):
    """Whatever the caller's TORCH_NCCL_CUDA_EVENT_CACHE (unset, or the cache explicitly on), the group the
    collectives are captured on is constructed with it "0", the caller's value is restored afterwards, and the
    group is built once per default group."""
    if caller_env is None:
        monkeypatch.delenv("TORCH_NCCL_CUDA_EVENT_CACHE", raising=False)
    else:
        monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", caller_env)
    seen = []
    sentinel = object()

    def fake_new_group(*a, **kw):
        seen.append((os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE"), kw.get("backend")))
        return sentinel

    monkeypatch.setattr(dist, "get_backend", lambda *a, **kw: "nccl")
    monkeypatch.setattr(dist, "new_group", fake_new_group)
    cvdist._CAPTURE_GROUP = None
    g = cvdist.captured_collectives_group()
    assert g is sentinel and seen == [("0", "nccl")]
    assert os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE") == caller_env
    assert cvdist.captured_collectives_group() is sentinel and len(seen) == 1  # cached


def test_buckets_use_the_given_group(gloo_world1, monkeypatch):
    """GradBuckets issues its all-reduces on the group it was given (the engine passes the dedicated one)."""
    import torch

    calls = []
    real = dist.all_reduce

    def spy(t, op=None, group=None, async_op=False):
        calls.append(group)
        return real(t, op=op, group=group, async_op=async_op)

    monkeypatch.setattr(dist, "all_reduce", spy)
    flat = torch.arange(6, dtype=torch.float32)
    grp = dist.new_group(backend="gloo")
    b = cvdist.GradBuckets(flat, [(3, 6), (0, 3)], group=grp, force=True)
    b.reduce_all()
    assert calls == [grp, grp]
    assert flat.tolist() == list(range(6))
