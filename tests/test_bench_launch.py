"""bench.py's launcher contract (CPU): `python bench.py --gpus N` starts N
ranks itself (one process per GPU, through torch.distributed.run) when no
launcher did, and never falls back to fewer GPUs silently. `--dry-launch`
makes each rank report its RANK/WORLD_SIZE and exit before touching a GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=300,
                          cwd=REPO)


def _objects(stdout):
    """Every JSON object in the stream, wherever the line breaks fall (each rank
    writes its line with one write(2), but the parser does not rely on it)."""
    dec = json.JSONDecoder()
    i, out = 0, []
    while True:
        i = stdout.find("{", i)
        if i < 0:
            return out
        try:
            d, i = dec.raw_decode(stdout, i)
            out.append(d)
        except ValueError:
            i += 1


def _ranks(stdout):
    return sorted((d["rank"], d["world_size"], d["local_rank"])
                  for d in _objects(stdout) if isinstance(d, dict) and d.get("dry_launch"))


def test_objects_parser_handles_interleaving():
    a, b = json.dumps({"dry_launch": True, "rank": 0}), json.dumps({"dry_launch": True, "rank": 1})
    assert [d["rank"] for d in _objects(a + b + "\nnoise {x\n" + a)] == [0, 1, 0]


@pytest.mark.parametrize("n", [2, 3, 8])
def test_gpus_n_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert _ranks(r.stdout) == [(k, n, k) for k in range(n)]


def test_gpus_1_runs_in_process():
    r = _run(["--gpus", "1", "--dry-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert _ranks(r.stdout) == [(0, 1, 0)]


def test_launcher_world_size_mismatch_fails():
    r = _run(["--gpus", "4", "--dry-launch"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_more_gpus_than_visible_fails():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    r = _run(["--gpus", str(n)])
    assert r.returncode != 0 and "visible" in r.stderr
