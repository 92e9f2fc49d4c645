"""Device RNG state for the reparameterisation noise and the CLUB-S permutation.

The reference draws eps with ``torch.randn_like`` (code/src/models/vae.py:59) and the CLUB-S
permutation with ``torch.randperm`` on the CPU generator (code/src/models/mi_estimator.py:138).
Here both come from a counter-based Philox4x32-10 stream on the device, keyed by
``torch.initial_seed()`` so ``torch.manual_seed(s)`` makes runs reproducible; the counter is a device
int64 advanced by the kernels themselves, so HIP-graph replays draw fresh noise.

Test hook (SURVEY 8b "RNG"): ``inject_noise([...])`` / ``inject_perm([...])`` queue explicit tensors
that the next ``sample()`` / CLUB-S calls consume instead of drawing, without any signature change.
"""

from __future__ import annotations

import collections

import torch

_state = {}
_noise_q: collections.deque = collections.deque()
_perm_q: collections.deque = collections.deque()


def offset_tensor(device) -> tuple[int, torch.Tensor]:
    """(seed, int64[2] device counter) for `device`; re-keyed when torch's seed changes."""
    device = torch.device(device)
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    seed = torch.initial_seed() & 0xFFFFFFFFFFFFFFFF
    st = _state.get(key)
    if st is None or st[0] != seed:
        st = (seed, torch.zeros(2, dtype=torch.int64, device=device))
        _state[key] = st
    return st


def reset_counters():
    """Restart every device's Philox stream at counter 0 (what a fresh process after
    torch.manual_seed(s) sees).  Engines and the module path share one counter per (device, seed), so
    consecutive engines draw fresh noise; call this to replay a stream from its start."""
    for _, off in _state.values():
        off.zero_()


def inject_noise(tensors):
    """Queue eps tensors (one per sample() call, shaped like its mu) for the next draws."""
    _noise_q.extend(tensors)


def inject_perm(perms):
    """Queue int64 permutations for the next CLUBSample.forward calls."""
    _perm_q.extend(perms)


def clear_injections():
    _noise_q.clear()
    _perm_q.clear()


def next_noise():
    return _noise_q.popleft() if _noise_q else None


def next_perm():
    return _perm_q.popleft() if _perm_q else None


def pending_noise() -> int:
    return len(_noise_q)
