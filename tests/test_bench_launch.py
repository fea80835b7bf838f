"""bench.py's rank launcher (CPU): `bench.py --gpus N` without a torchrun environment starts N data-parallel ranks
itself, every rank joins one process group of the launched size, and exactly one line (rank 0's) reports the live
world size.  Under a launcher, WORLD_SIZE must equal --gpus.  The GPU half (the real step over gloo on one GPU) is
tests/test_bench_gpu.py::test_bench_ranks_gloo."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def test_bench_launches_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-selftest"], capture_output=True, text=True,
                       timeout=300, cwd=ROOT, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["parallelism"] == "dp3" and d["rank_sum"] == 0 + 1 + 2


def test_bench_world_size_must_match_gpus():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-selftest"], capture_output=True, text=True,
                       timeout=120, cwd=ROOT, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in r.stderr


def test_bench_single_rank_needs_no_launcher():
    r = subprocess.run([sys.executable, BENCH, "--launch-selftest"], capture_output=True, text=True, timeout=120,
                       cwd=ROOT, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["parallelism"] == "dp1"
