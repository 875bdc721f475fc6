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
