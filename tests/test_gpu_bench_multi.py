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


def _run(extra_env=None, args=()):
    env = dict(os.environ, TRPO_BENCH_DEVICE="0", **(extra_env or {}))
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                        "--warmup", "3", "--no-extra", *args],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), r.stderr


def _self_checked(d):
    """the N > 1 line carries the collective's self-check, the cross-rank x-hash
    agreement and the sharded step's parity against the reference CG on the whole batch."""
    v = d["comm"]["verify"]
    assert v["eager_allreduce_exact"] and v["x_identical_on_all_ranks"] and len(v["x_sha256_16"]) == 16
    assert d["parity"]["cg_step_relL2_vs_cpu"] <= 1e-4, d["parity"]


def test_bench_two_ranks_one_gpu_prints_one_line():
    d, _ = _run()
    assert d["n_gpus"] == 2 and d["comm"]["ranks"] == 2
    assert d["config"]["samples"] == 50_000 and d["config"]["samples_per_rank"] == 25_000
    assert d["value"] > 0 and d["ms_per_step"] > 0
    fb = d["comm"]["fallback"]
    if fb is not None:                               # RCCL refused the shared device
        assert fb["requested"] == "rccl" and d["comm"]["backend"].startswith("peer")
        assert "peer-window" in d["config"]["parallelism"]
    _self_checked(d)


def test_bench_two_ranks_forced_verify_failure_falls_back():
    """The library's self-check made to fail on rank 1 in the first attempt (TRPO_COMM_FAULT via
    TRPO_BENCH_FAULT=comm-verify:1): both ranks see a wrong exact sum, abort, try RCCL (refused on one
    device), then the peer exchange again -- one JSON line, exit 0, the failures recorded."""
    d, err = _run({"TRPO_BENCH_FAULT": "comm-verify:1"}, ("--comm", "peer"))
    fb = d["comm"]["fallback"]
    assert fb["requested"] == "peer", fb
    assert fb["failed"][0]["stage"] == "verify" and fb["failed"][0]["comm"] == "peer", fb
    assert d["comm"]["backend"].startswith("peer") and d["comm"]["verify"]["attempt"] >= 1
    _self_checked(d)


def test_bench_two_ranks_hung_rank_is_bounded():
    """Rank 1 skips the self-check's all-reduce (comm-hang:1): rank 0's exchange gives up after its 3-s
    bound, every rank aborts and moves on; the run still ends with one verified line."""
    d, _ = _run({"TRPO_BENCH_FAULT": "comm-hang:1"}, ("--comm", "peer", "--no-cpu-baseline"))
    fb = d["comm"]["fallback"]
    assert fb["failed"][0]["stage"] == "verify", fb
    assert d["comm"]["verify"]["x_identical_on_all_ranks"]
