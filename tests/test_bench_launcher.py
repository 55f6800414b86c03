"""bench.py --gpus N launches N ranks.

CPU: ``--plumbing`` runs the same launcher path (plain ``python bench.py --gpus 2`` ->
torch.distributed.run -> 2 processes) with a gloo group instead of RCCL and no GPU work;
rank 0 reports the world size it joined.  A WORLD_SIZE that disagrees with ``--gpus`` is
refused with a non-zero exit."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=300)


def test_launcher_spawns_two_ranks():
    r = _run(["--gpus", "2", "--plumbing"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2 and rec["requested"] == 2
    assert rec["backend"] == "gloo"


def test_launcher_single_rank_no_spawn():
    r = _run(["--gpus", "1", "--plumbing"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0",
                                             "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29533"})
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 1 and rec["ranks_seen"] == 1


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "4", "--plumbing"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
