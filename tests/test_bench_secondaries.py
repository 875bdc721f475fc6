"""CPU: bench.py's N > 1 path end to end as TWO real processes over gloo, the device library replaced
by fake contexts (tests/bench_fake_rank.py), with one-sided faults injected into the secondary
configs that run after the headline: a context that fails to build on one rank (an
OOM at a sweep row), a failed agreed setup stage, a solve that fails inside the timed region, and a
rank that blocks forever inside a secondary (a library call ignoring its bound).  Every case must end
in bounded time with exit 0 and exactly one JSON line whose headline is intact and whose failed
secondaries are recorded as errors."""
import json
import os
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run2(fault=None, env_extra=None, args=("--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--comm", "rccl"),
          limit=150):
    # (--comm rccl: the scenario these cases were written for -- RCCL headline, the peer forms as secondaries;
    # the default collective is the peer exchange since round 6, which the fake context serves the same way)
    port = _port()
    procs = []
    t0 = time.monotonic()
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TRPO_GLOO_SECONDARY_TIMEOUT_S="6", TRPO_BENCH_DEADLINE_S="20",
                   TRPO_BENCH_GRACE_S="5", **(env_extra or {}))
        env.pop("TRPO_BENCH_FAULT", None)
        if fault:
            env["TRPO_BENCH_FAULT"] = fault
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "bench_fake_rank.py"), "--gpus", "2", *args],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=limit))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    wall = time.monotonic() - t0
    for p, (_, err) in zip(procs, outs):
        assert p.returncode == 0, err[-3000:]
    assert outs[1][0] == "", outs[1][0]                     # rank 1 prints nothing on stdout
    lines = outs[0][0].splitlines()
    assert len(lines) == 1, outs[0][0]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["comm"]["verify"]["x_identical_on_all_ranks"]
    return d, wall, outs


def _ok(row):
    return isinstance(row, dict) and "error" not in row


def test_secondaries_all_run_without_faults():
    d, _, _ = _run2()
    assert "dist_broken" not in d
    ex = d["extra"]
    for k in ("C4_peer_exchange", "C4_peer_flag_exchange", "C5_update_armDOF_0_N50000"):
        assert _ok(ex[k]), (k, ex[k])
    assert ex["C4_peer_exchange"]["verify"]["x_identical_on_all_ranks"]
    sw = ex["C4_sweep"]
    assert set(sw) == {"cg10_armDOF_0_N4000", "cg10_armDOF_0_N6000", "cg10_armDOF_0_N100000"}
    assert all(_ok(r) for r in sw.values()), sw
    assert sw["cg10_armDOF_0_N100000"]["scaling"].startswith("weak")
    assert "watchdog" not in d


def test_sweep_context_fails_on_one_rank():
    """A sweep row's context fails on rank 1 only (e.g. out of memory at the large row): both ranks
    record the row as failed at stage `context`, and the remaining rows still run."""
    d, _, _ = _run2("sweep4000.context:1")
    sw = d["extra"]["C4_sweep"]
    assert "error" in sw["cg10_armDOF_0_N4000"] and "context" in sw["cg10_armDOF_0_N4000"]["error"]
    assert _ok(sw["cg10_armDOF_0_N6000"]) and _ok(sw["cg10_armDOF_0_N100000"])
    assert _ok(d["extra"]["C5_update_armDOF_0_N50000"])


def test_update_setup_and_solve_fail_on_one_rank():
    """The update's agreed setup fails at `solve` on rank 1, then in a second run its updates fail on
    rank 1: the update row is an error on rank 0 too, and the sweep after it is complete."""
    d, _, _ = _run2("update.solve:1")
    up = d["extra"]["C5_update_armDOF_0_N50000"]
    assert "error" in up and "solve" in up["error"], up
    assert all(_ok(r) for r in d["extra"]["C4_sweep"].values())
    d, _, outs = _run2("update.update:1")
    err0 = outs[0][1]
    up = d["extra"]["C5_update_armDOF_0_N50000"]
    assert "error" in up and "another rank failed at update.update" in up["error"], up
    assert "fake: comm_abort" in err0                       # the failed secondary's collective was aborted
    assert all(_ok(r) for r in d["extra"]["C4_sweep"].values())


def test_sweep_timed_region_fails_on_one_rank():
    d, _, _ = _run2("sweep6000.timed:1")
    sw = d["extra"]["C4_sweep"]
    assert "error" in sw["cg10_armDOF_0_N6000"], sw
    assert _ok(sw["cg10_armDOF_0_N4000"]) and _ok(sw["cg10_armDOF_0_N100000"])


def test_hung_rank_in_a_secondary_is_bounded():
    """Rank 1 blocks forever inside the update secondary: rank 0's next agreement times out on the
    secondary gloo group (6 s here), the remaining secondaries are skipped, rank 0 prints the line; rank
    1's watchdog ends it at the deadline.  Both exit 0, well inside the limit."""
    d, wall, _ = _run2("update.hang:1")
    assert d.get("dist_broken") is True                    # the line says a secondary's collective failed
    ex = d["extra"]
    assert _ok(ex["C4_peer_exchange"])
    assert "error" in ex["C5_update_armDOF_0_N50000"]
    assert "C4_sweep" not in ex or all("error" in r for r in ex["C4_sweep"].values())
    assert wall < 90


def test_hung_rank0_prints_by_watchdog():
    """Rank 0 itself blocks inside a secondary: its watchdog prints the headline line (marked) at the
    deadline and ends the process with exit 0."""
    d, wall, _ = _run2("flag.hang:0")
    assert "deadline reached" in d["watchdog"]
    assert _ok(d["extra"]["C4_peer_exchange"])
    assert "C4_peer_flag_exchange" not in d["extra"]
    assert wall < 90


def test_default_collective_is_the_peer_exchange():
    """Round 6: without --comm the headline's collective is the peer-window exchange, and RCCL is the
    measured secondary (extra.C4_rccl_exchange) beside the flag form and the sharded update."""
    d, _, _ = _run2(args=("--steps", "3", "--warmup", "1", "--no-cpu-baseline"))
    assert d["comm"]["backend"] == "peer" and "peer-window" in d["config"]["parallelism"]
    ex = d["extra"]
    for k in ("C4_rccl_exchange", "C4_peer_flag_exchange", "C5_update_armDOF_0_N50000"):
        assert _ok(ex[k]), (k, ex[k])
    assert ex["C4_rccl_exchange"]["backend"] == "rccl"
