"""Worker of tests/test_dist_gloo.py (importable by spawned processes)."""

import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "clear-vae_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def run(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(2)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from cvhip import dist as cvd

        out = {}
        # bucketed async SUM all-reduce over contiguous views of one flat arena (decoder bucket first)
        flat = torch.arange(10, dtype=torch.float64) * (rank + 1)
        b = cvd.GradBuckets(flat, [(6, 10), (0, 6)])
        b.launch(0)
        b.launch(1)
        b.wait()
        out["buckets"] = flat.tolist()
        # construction-time broadcast of rank 0's parameters
        p = torch.full((5,), float(rank + 7))
        cvd.broadcast_flat(p)
        out["broadcast"] = p.tolist()
        # DDP semantics on the oracle: rank r computes the CLEAR step on its shard of the global batch,
        # the flat gradient is averaged through the same reduction the engine uses
        from oracle import cpu_ref as R

        n_global = 24
        x, label, ec, es, _ = R.det_inputs(n_global, 1, 28, 16, 4, seed=11)
        lo, hi = cvd.shard_bounds(n_global, rank, world)
        P = R.to_torch(R.det_state("VAE", 16, 1))
        hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "ps": True}
        o = R.clear_step(P, torch.tensor(x[lo:hi]), torch.tensor(label[lo:hi]), torch.tensor(ec[lo:hi]),
                         torch.tensor(es[lo:hi]), "VAE", hp)
        g = torch.cat([v.reshape(-1) for v in o["grads"].values()]).detach()
        cvd.average_in_place(g)
        out["grad"] = g.numpy()
        out["bounds"] = (lo, hi)
        dist.destroy_process_group()
        q.put((rank, out, None))
    except Exception:  # pragma: no cover
        q.put((rank, None, traceback.format_exc()))
