"""bench.py's output contract (the driver parses it): one JSON line with the required keys, the whole-job
value consistent with ms_per_step, and the roofline / cpu_baseline objects filled from live measurements."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


@pytest.mark.parametrize("config", ["cfg2", "cfg4"])
def test_bench_json_line(config):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", config, "--steps", "6",
                        "--warmup", "2", "--cpu-baseline-seconds", "0.5"], capture_output=True, text=True,
                       timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert REQUIRED <= set(d), REQUIRED - set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 6 and d["scaling"] == "weak" and d["higher_is_better"] is True
    B = d["config"]["per_gpu_batch"]
    assert abs(d["value"] - B / (d["ms_per_step"] * 1e-3)) < 0.01 * d["value"]
    roof = d["roofline"]
    assert roof["live_samples"] == 2 * 6                      # 2 layers' attention backward x 6 timed steps
    assert roof["bound"] in ("hbm", "mfma") and 0 < roof["frac"] < 1 and roof["peak"] > 0
    assert 0.5 < roof["avg_launch_us"] / roof["isolated_launch_us"] < 2.0
    cpu = d["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["value"] > 0 and cpu["cores"] >= 1


@pytest.mark.parametrize("n", [2, 8])
def test_bench_ranks_gloo(n):
    """`bench.py --gpus N` started alone launches its data-parallel ranks itself (here: N processes on one GPU over
    gloo, N = 8 the scaling run's rank count; the driver's SCALE runs use RCCL on one GPU per rank): one JSON line,
    the live world size, the replicas' parameters equal after the warmup steps, the whole-job value over all ranks."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dist-backend", "gloo",
                        "--config", "cfg2", "--steps", "4", "--warmup", "2", "--roofline-replays", "2"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert REQUIRED <= set(d), REQUIRED - set(d)
    assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}" and d["config"]["global_batch"] == 128 * n
    assert d["dp"]["replicas_equal_after_warmup"] is True and d["dp"]["backend"] == "gloo"
    assert abs(d["value"] - 128 * n / (d["ms_per_step"] * 1e-3)) < 0.01 * d["value"]
    assert d["cpu_baseline"] is None                          # rank 0 at N = 1 only
