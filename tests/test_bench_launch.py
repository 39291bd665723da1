"""bench.py --gpus N without torchrun starts N ranks itself (CPU/gloo self-test of the
launcher; the GPU path uses the same spawn with RCCL)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--selftest-dist"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_spawns_requested_ranks():
    r = _run(2)
    assert r["n_gpus"] == 2 and r["rank_sum"] == 3.0


def test_bench_single_rank():
    assert _run(1)["n_gpus"] == 1


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--selftest-dist"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr
