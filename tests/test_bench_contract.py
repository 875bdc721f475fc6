"""CPU: bench.py's roofline accounting (SURVEY §8d per-sample figures) and its launch contract."""
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_per_sample_figures_armdof0():
    b = _bench()
    L = [15, 16, 16, 3]
    assert b.num_params(L) == 582
    assert b.flops_per_sample(L) == 4710            # SURVEY §8a recompute FVP
    assert b.flops_per_sample_cached(L) == 3622     # forward cached across the solve's FVPs
    # observations + cached y1, y2 in fp32 per sample; theta, v, Fv per launch
    assert b.bytes_per_fvp_cached(L, 50_000) == 188 * 50_000 + 12 * 582
    assert b.bytes_cg_step(L) == 64 * 582
    # the headline roofline's algorithmic bytes per CG-iteration launch (9.44 MB)
    assert b.bytes_per_fvp_cached(L, 50_000) + b.bytes_cg_step(L) == 9_444_232


def test_rank_count_mismatch_exits_nonzero():
    """Under a launcher whose WORLD_SIZE differs from --gpus the bench refuses to run (exit 2)
    instead of timing a different configuration; this check runs before anything touches a GPU."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


class _FakeDist:
    """Two ranks seen from rank 0.  `other_fails` = {(attempt, stage)}: the OTHER rank reports a failure
    at that stage of that attempt (the agreement after the stage then fails on every rank)."""

    def __init__(self, other_fails=()):
        self.world, self.rank, self.other_fails = 2, 0, set(other_fails)
        self.attempt, self.stage_i = -1, 0
        self.calls = []

    def max(self, x):
        import bench_mod
        st = bench_mod.STAGES[min(self.stage_i, len(bench_mod.STAGES) - 1)]
        self.stage_i += 1
        self.calls.append(st)
        return max(x, 1.0 if (self.attempt, st) in self.other_fails else 0.0)

    def allgather_bytes(self, b):
        return [b, b]

    def bcast_bytes(self, b):
        return b if b is not None else b"uid"


class _FakeCtx:
    made = []

    def __init__(self, *a, **k):
        self.closed, self.aborted, self.backend, self.attach_kw = False, False, None, None
        _FakeCtx.made.append(self)

    def peer_handle(self):
        return b"h" * 64

    def attach_peers(self, rank, world, handles):
        self.backend = "peer"

    def attach_comm(self, rank, world, uid, timeout_ms=0):
        self.backend, self.attach_kw = "rccl", timeout_ms

    def comm_info(self):
        return dict(rank=0, world=2, replicas=2, backend=self.backend)

    def comm_verify(self, timeout_ms=0):
        pass

    def upload_b(self, b):
        pass

    def enqueue_cg(self, *a):
        pass

    def wait(self, timeout_ms=0):
        pass

    def download_x(self):
        import numpy as np
        return np.arange(582, dtype=np.float64)

    def comm_abort(self):
        self.aborted = True

    def close(self):
        self.closed = True


def _agreed(monkeypatch, other_fails=(), comm="rccl", fault=None, local_fails=None):
    """Run make_ctx_agreed with fake contexts; local_fails = {(attempt, stage)} raised on THIS rank."""
    import numpy as np
    import trpo_amd
    from trpo_amd import synth  # noqa: F401 -- the real seeded synthesis
    b = _bench()
    sys.modules["bench_mod"] = b
    dist = _FakeDist(other_fails)
    _FakeCtx.made = []
    local_fails = set(local_fails or ())

    class Ctx(_FakeCtx):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            if (dist.attempt, "context") in local_fails:
                raise trpo_amd.TRPOError("trpo_ctx_create failed")

        def attach_comm(self, *a):
            if (dist.attempt, "attach") in local_fails:
                raise trpo_amd.TRPOError("attach_comm failed (-4)")
            super().attach_comm(*a)

        def attach_peers(self, *a):
            if (dist.attempt, "attach") in local_fails:
                raise trpo_amd.TRPOError("attach_peers failed (-4)")
            super().attach_peers(*a)

        def comm_verify(self, timeout_ms=0):
            if (dist.attempt, "verify") in local_fails:
                raise trpo_amd.TRPOError("comm_verify failed (-7)")
            super().comm_verify(timeout_ms)

    monkeypatch.setattr(trpo_amd, "Context", Ctx)
    monkeypatch.setattr(trpo_amd, "unique_id", lambda: b"u" * 128)
    orig = b.make_ctx_agreed.__globals__["_fault"]

    def fault_hook(stage, rank, attempt):
        if stage == "context":               # first check of every attempt: track the attempt number
            dist.attempt, dist.stage_i = attempt, 0
        return orig(stage, rank, attempt)

    monkeypatch.setitem(b.make_ctx_agreed.__globals__, "_fault", fault_hook)
    if fault:
        monkeypatch.setenv("TRPO_BENCH_FAULT", fault)
    else:
        monkeypatch.delenv("TRPO_BENCH_FAULT", raising=False)
    out = b.make_ctx_agreed([15, 16, 16, 3], 64, dist, 0, comm, np.ones(582))
    return b, dist, _FakeCtx.made, out


def test_headline_collective_agreed_no_fallback(monkeypatch):
    _, dist, made, (ctx, _, _, used, rec) = _agreed(monkeypatch)
    assert used == "rccl" and rec["fallback"] is None and ctx is made[0] and not ctx.closed
    v = rec["verify"]
    assert v["eager_allreduce_exact"] and v["x_identical_on_all_ranks"] and len(v["x_sha256_16"]) == 16
    # one agreement per stage, plus the x-hash comparison
    assert dist.calls == ["context", "bootstrap", "attach", "verify", "solve", "hash", "hash"]


def test_headline_falls_back_when_this_rank_fails_attach(monkeypatch):
    """RCCL refusing to attach (e.g. two ranks on one device) moves every rank to the peer exchange."""
    _, _, made, (ctx, _, _, used, rec) = _agreed(monkeypatch, local_fails={(0, "attach")})
    assert used == "peer" and ctx.backend == "peer" and made[0].closed and not made[0].aborted
    fb = rec["fallback"]
    assert fb["requested"] == "rccl" and fb["failed"][0]["stage"] == "attach"
    assert "attach_comm failed" in fb["failed"][0]["error"]


def test_headline_falls_back_when_another_rank_fails(monkeypatch):
    """This rank attached but another did not: its collective is aborted, its context closed, and it
    moves on with the others."""
    _, _, made, (ctx, _, _, used, rec) = _agreed(monkeypatch, other_fails={(0, "attach")})
    assert used == "peer" and made[0].closed and not ctx.closed
    assert made[0].aborted                    # it had attached: abort before close
    assert rec["fallback"]["failed"][0]["error"] == "another rank failed at stage attach"


def test_one_sided_failure_at_every_stage_is_agreed(monkeypatch):
    """a failure on ONE rank at any stage makes every rank leave together."""
    b = _bench()
    for st in b.STAGES:
        _, _, made, (ctx, _, _, used, rec) = _agreed(monkeypatch, other_fails={(0, st)})
        assert used == "peer", st
        assert rec["fallback"]["failed"][0]["stage"] == st
        assert made[0].closed


def test_verify_failure_aborts_and_retries(monkeypatch):
    """A failed self-check (wrong sum or time-out) aborts the collective on every rank; with both
    backends failing once the third attempt (the requested one again) carries the headline."""
    _, _, made, (ctx, _, _, used, rec) = _agreed(monkeypatch, local_fails={(0, "verify"), (1, "attach")})
    assert used == "rccl" and len(made) == 3
    assert made[0].aborted and made[0].closed and made[1].closed and not ctx.closed
    assert [f["stage"] for f in rec["fallback"]["failed"]] == ["verify", "attach"]
    assert rec["verify"]["attempt"] == 2


def test_fault_injection_env(monkeypatch):
    """TRPO_BENCH_FAULT=<stage>:<rank>[:<attempt>] (the knob the 2-rank GPU test uses)."""
    _, _, made, (ctx, _, _, used, rec) = _agreed(monkeypatch, fault="solve:0")
    assert used == "peer" and made[0].aborted
    assert rec["fallback"]["failed"][0]["stage"] == "solve"
    assert "injected" in rec["fallback"]["failed"][0]["error"]
    _, _, made, (ctx, _, _, used, rec) = _agreed(monkeypatch, fault="hash-mismatch:0")
    assert used == "peer" and rec["fallback"]["failed"][0]["stage"] == "hash"


def test_library_fault_is_armed_for_one_attempt_only(monkeypatch):
    """comm-verify:R sets TRPO_COMM_FAULT=verify:R (read by the library's self-check) during attempt 0
    only, and leaves the environment as it was afterwards."""
    import os
    seen = []
    b = _bench()

    def spy(*a, **k):
        seen.append(os.environ.get("TRPO_COMM_FAULT"))

    monkeypatch.setattr(_FakeCtx, "comm_verify", lambda self, t=0: spy())
    _agreed(monkeypatch, fault="comm-verify:0")
    assert seen == ["verify:0"]
    assert "TRPO_COMM_FAULT" not in os.environ


def test_headline_exits_when_no_collective_passes(monkeypatch):
    import pytest
    with pytest.raises(SystemExit):
        _agreed(monkeypatch, local_fails={(0, "attach"), (1, "attach"), (2, "attach")})


def test_pmc_median_per_dispatch(tmp_path):
    """roofline.traffic's parser (bench.pmc_median): per-dispatch totals over counter instances, the
    median over the CG-iteration kernel's dispatches only; None when no dispatch matches."""
    import bench
    p = tmp_path / "run_counter_collection.csv"
    rows = ["Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value"]
    k3 = "void fvp_mlp3_kernel<1, 1, 1, 1, 5, 3, 4, 11>(double const*)"
    for d, vals in ((1, (100.0, 20.0)), (2, (110.0, 20.0)), (3, (500.0, 0.0))):
        for v in vals:
            rows.append('%d,"%s",FETCH_SIZE,%s' % (d, k3 if d < 3 else "cg_last_kernel(double const*)", v))
    rows.append('4,"%s",WRITE_SIZE,7.0' % k3)
    p.write_text("\n".join(rows) + "\n")
    assert bench.pmc_median(str(p), "FETCH_SIZE") == (125.0, 2)
    assert bench.pmc_median(str(p), "WRITE_SIZE") == (7.0, 1)
    assert bench.pmc_median(str(p), "FETCH_SIZE", kernel="no such kernel") is None


def test_measure_traffic_without_profiler(monkeypatch):
    """No rocprofv3 on the host: measure_traffic reports why and the bench falls back (no exception)."""
    import shutil
    import bench
    monkeypatch.setattr(shutil, "which", lambda name: None)
    monkeypatch.setattr(bench.os.path, "exists", lambda p: False)
    assert bench.measure_traffic(0) == (None, "rocprofv3 not found")


def test_mfma_busy_from_counters():
    """roofline.mfma_busy_frac: SQ_VALU_MFMA_BUSY_CYCLES (summed over every SIMD) over
    1 024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs.  Round 5's committed counters of the 50k kernel
    (profiles/r05_sq_counters_cgiter.txt: 3.0 M busy cycles, ~9 us at ~2.3 GHz) read ~14 %; a dispatch
    whose every SIMD issued MFMAs for its whole active time reads 1."""
    import bench
    med = {"SQ_VALU_MFMA_BUSY_CYCLES": (3.0e6, 9), "SQ_INSTS_MFMA": (112500.0, 9), "SQ_BUSY_CYCLES": (624725.0, 9),
           "SQ_WAVE_CYCLES": (9.04e6, 9), "SQ_WAIT_INST_ANY": (2.65e6, 9), "GRBM_GUI_ACTIVE": (8 * 20700.0, 9)}
    m = bench.mfma_from_counters(med)
    assert abs(m["mfma_busy_frac"] - 3.0e6 / (1024 * 20700.0)) < 1e-12
    assert 0.13 < m["mfma_busy_frac"] < 0.15
    assert abs(m["wait_inst_any_frac"] - 2.65e6 / 9.04e6) < 1e-12
    assert m["dispatches"] == 9 and "GRBM_GUI_ACTIVE" in m["mfma_busy_denominator"]
    assert "mfma_busy_frac_at_peak_clock" not in m
    m = bench.mfma_from_counters(med, kernel_ms=0.009)              # 9 us at 2.4 GHz = 21 600 cycles
    assert abs(m["mfma_busy_frac_at_peak_clock"] - 3.0e6 / (1024 * 21600.0)) < 1e-12
    assert m["mfma_busy_frac"] == m["mfma_busy_frac_at_peak_clock"]          # the event form leads when known
    assert abs(m["mfma_busy_frac_grbm"] - 3.0e6 / (1024 * 20700.0)) < 1e-12
    full = dict(med, SQ_VALU_MFMA_BUSY_CYCLES=(1024 * 20700.0, 9))
    assert abs(bench.mfma_from_counters(full)["mfma_busy_frac"] - 1.0) < 1e-12


def test_measure_mfma_without_profiler(monkeypatch):
    """No rocprofv3: measure_mfma returns the reason, no exception (the line then carries null)."""
    import shutil
    import bench
    monkeypatch.setattr(shutil, "which", lambda name: None)
    monkeypatch.setattr(bench.os.path, "exists", lambda p: False)
    assert bench.measure_mfma(0) == {"error": "rocprofv3 not found"}
    assert bench.measure_mfma(0, 4_000_000) == {"error": "rocprofv3 not found"}
