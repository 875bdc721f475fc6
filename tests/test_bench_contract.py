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
    """Two ranks seen from rank 0; `peer_fails` = backends whose attach fails on the OTHER rank."""

    def __init__(self, peer_fails=()):
        self.world, self.rank, self.peer_fails, self.current = 2, 0, set(peer_fails), None

    def max(self, x):
        return max(x, 1.0 if self.current in self.peer_fails else 0.0)


class _FakeCtx:
    def __init__(self, comm):
        self.comm, self.closed = comm, False

    def close(self):
        self.closed = True


def _agreed(monkeypatch, local_fails=(), peer_fails=(), comm="rccl"):
    b = _bench()
    dist = _FakeDist(peer_fails)
    made = []

    def fake_make_ctx(L, n, d, device, comm="rccl"):
        dist.current = comm
        if comm in local_fails:
            raise RuntimeError("attach_%s failed (-4)" % comm)
        made.append(_FakeCtx(comm))
        return made[-1], "theta", "obs"

    monkeypatch.setattr(b, "make_ctx", fake_make_ctx)
    return b, dist, made, b.make_ctx_agreed(b.ARM, b.N_TOTAL, dist, 0, comm)


def test_headline_collective_agreed_no_fallback(monkeypatch):
    _, _, made, (ctx, _, _, used, fb) = _agreed(monkeypatch)
    assert used == "rccl" and fb is None and ctx is made[0] and not ctx.closed


def test_headline_falls_back_when_this_rank_fails(monkeypatch):
    """RCCL refusing to attach (e.g. two ranks on one device) moves every rank to the peer exchange."""
    _, _, made, (ctx, _, _, used, fb) = _agreed(monkeypatch, local_fails={"rccl"})
    assert used == "peer" and ctx.comm == "peer"
    assert fb["requested"] == "rccl" and "attach_rccl failed" in fb["failed"][0]["error"]


def test_headline_falls_back_when_another_rank_fails(monkeypatch):
    """This rank attached but another did not: its context is closed and it moves on with the others."""
    _, _, made, (ctx, _, _, used, fb) = _agreed(monkeypatch, peer_fails={"rccl"})
    assert used == "peer" and made[0].closed and not ctx.closed
    assert fb["failed"][0]["error"] == "another rank failed to attach"


def test_headline_exits_when_no_collective_attaches(monkeypatch):
    import pytest
    with pytest.raises(SystemExit):
        _agreed(monkeypatch, local_fails={"rccl", "peer"})
