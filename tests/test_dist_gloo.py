"""Data-parallel path on CPU: world_size-2 gloo processes exercise cvhip/dist.py exactly as the
engine uses it (broadcast of rank 0's arena, bucketed async SUM all-reduce, 1/world averaging), and
check that the DP step has DDP semantics: the averaged gradient equals the mean of the per-shard
oracle gradients computed in one process."""

import multiprocessing as mp
import socket

import numpy as np
import torch

import dp_worker


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(world=2, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=dp_worker.run, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, out, err = q.get(timeout=timeout)
            assert err is None, err
            res[r] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


def test_world2_gloo():
    from cvhip import dist as cvd
    from oracle import cpu_ref as R

    res = _launch()
    want = (np.arange(10) * 3.0).tolist()
    for r in (0, 1):
        assert res[r]["buckets"] == want
        assert res[r]["broadcast"] == [7.0] * 5
    # shards tile the global batch
    assert res[0]["bounds"] == (0, 12) and res[1]["bounds"] == (12, 24)
    assert cvd.shard_bounds(25, 1, 2) == (13, 25)
    # both ranks hold the same averaged gradient ...
    assert np.array_equal(res[0]["grad"], res[1]["grad"])
    # ... equal to the mean of the per-shard gradients (DDP semantics)
    x, label, ec, es, _ = R.det_inputs(24, 1, 28, 16, 4, seed=11)
    hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "ps": True}
    gs = []
    for lo, hi in ((0, 12), (12, 24)):
        P = R.to_torch(R.det_state("VAE", 16, 1))
        o = R.clear_step(P, torch.tensor(x[lo:hi]), torch.tensor(label[lo:hi]), torch.tensor(ec[lo:hi]),
                         torch.tensor(es[lo:hi]), "VAE", hp)
        gs.append(torch.cat([v.reshape(-1) for v in o["grads"].values()]).detach().numpy())
    ref = (gs[0] + gs[1]) / 2
    # (absolute floor: biases feeding a train-mode BN have rounding-noise gradients that depend on the
    # CPU thread count)
    assert np.allclose(res[0]["grad"], ref, rtol=1e-9, atol=1e-10 * np.abs(ref).max())
