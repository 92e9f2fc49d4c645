"""bench.py's rank launch (the multi-GPU contract): `python bench.py --gpus N` run directly starts
torch.distributed.run with N ranks as a child process, and rank 0 prints one line with n_gpus = N; under an
external launcher WORLD_SIZE must equal --gpus.  Checked with --dry-run (gloo, no GPU) so it runs here."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def _lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_gpus2_spawns_two_ranks():
    p = _run(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    recs = _lines(p.stdout)
    assert len(recs) == 1, p.stdout  # rank 0 only
    assert recs[0]["n_gpus"] == 2 and recs[0]["world_seen"] == 2


def test_gpus1_single_process():
    p = _run(["--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert _lines(p.stdout) == [{"dry_run": True, "n_gpus": 1, "world_seen": 1, "gpus_arg": 1}]


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
