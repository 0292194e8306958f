"""bench.py starts its own ranks when the driver runs `python bench.py --gpus N` without a
launcher (BASELINE "1/2/4/8 MI355X"): CPU-only rank plumbing (gloo), no GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.join(os.path.dirname(__file__), "..")


def run_bench(*args, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_self_launch_ranks(n):
    p = run_bench("--gpus", str(n), "--check-launch")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout   # ONE JSON line, from rank 0
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks"] == n and out["rank_sum"] == n * (n - 1) // 2
    assert out["local_rank"] == 0
    assert out["launcher"] == ("bench.py" if n > 1 else None)


def test_self_launch_failing_rank_ends_job():
    p = run_bench("--gpus", "2", "--check-launch", "--check-launch-fail-rank", "1", timeout=120)
    assert p.returncode != 0
    assert "rank 1 exited" in p.stderr
