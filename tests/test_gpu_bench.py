"""bench.py's own launch path: `--gpus N` without a torch.distributed launcher starts N rank processes (one per
GPU; here gloo with every rank on cuda:0, the rehearsal form) and rank 0 prints one JSON line whose n_gpus is the
process group's size."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(400)
def test_bench_gpus2_spawns_two_ranks():
    cmd = [sys.executable, "-u", "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--one-device", "--steps", "5",
           "--warmup", "2", "--no-cpu-baseline", "--no-train-loop", "--no-tcsr", "--only"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=360)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 400
    assert out["value"] > 0 and out["config"]["sampled_edges_per_step"] > 0
    assert "spawned 2 rank processes" in r.stderr
