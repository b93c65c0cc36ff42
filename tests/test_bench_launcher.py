"""bench.py's multi-GPU launcher on CPU (gloo): ``--gpus N`` with no
WORLD_SIZE starts N ranks itself; the shard split, the barrier and the
max-over-ranks timing run with no GPU work (``--dry-run``).  The real run
differs only in the backend (RCCL) and the per-rank GPU step."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=e, cwd=REPO)


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_self_launch_two_ranks():
    r = _bench("--gpus", "2", "--dry-run", "--steps", "2")
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["global_batch"] == 32
    assert line["shards"] == [[0, 16], [16, 16]]


def test_self_launch_c4_shape():
    """C4: 128 clouds over 8 ranks, 16 each, contiguous."""
    r = _bench("--gpus", "8", "--dry-run", "--steps", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 8 and line["global_batch"] == 128
    assert line["shards"] == [[16 * i, 16] for i in range(8)]


def test_world_size_must_match_gpus():
    r = _bench("--gpus", "2", "--dry-run", env={"WORLD_SIZE": "1"})
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
