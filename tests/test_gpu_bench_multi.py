"""MI355X: bench.py's N > 1 path end to end on ONE GPU (the driver's multi-GPU scaling run takes the
same code across GPUs).  `bench.py --gpus 2` launches its two rank processes itself; TRPO_BENCH_DEVICE=0
puts both on device 0, where RCCL refuses a second rank on the same device, so the headline's
collective agreement falls back to the peer-window exchange on both ranks (or stays on RCCL if a
future RCCL accepts it).  Checked: exit 0, exactly one line on stdout and it is the JSON line, two
ranks, the sharded solve's samples, and the collective actually used named in the line.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_one_gpu_prints_one_line():
    env = dict(os.environ, TRPO_BENCH_DEVICE="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                        "--warmup", "3", "--no-extra", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["comm"]["ranks"] == 2
    assert d["config"]["samples"] == 50_000 and d["config"]["samples_per_rank"] == 25_000
    assert d["value"] > 0 and d["ms_per_step"] > 0
    fb = d["comm"]["fallback"]
    if fb is not None:                               # RCCL refused the shared device
        assert fb["requested"] == "rccl" and d["comm"]["backend"].startswith("peer")
        assert "peer-window" in d["config"]["parallelism"]
