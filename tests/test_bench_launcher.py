"""``bench.py --gpus N`` launches N rank processes itself when no torchrun environment is set
(the driver's scaling runs call it either way).  CPU check: ``--dry-run`` ranks join a gloo group
and rank 0 reports the ranks the collective layer saw; no CUDA call is made."""

import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout        # exactly one JSON line, from rank 0
    return json.loads(lines[0])


def test_self_launch_two_ranks():
    out = _run(["--gpus", "2", "--dry-run", "--mode", "train"])
    assert out["n_gpus"] == 2 and out["ranks_seen"] == [0, 1] and out["mode"] == "train"


def test_single_rank_dry_run():
    out = _run(["--dry-run"])
    assert out["n_gpus"] == 1 and out["ranks_seen"] == [0]
