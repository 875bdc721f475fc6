"""Host-visible time of one baseline evaluate (the liblbfgs callback's device part) on the trainer's
[16,16,16,1] baseline and 20 x 150 batch, in a tight ctypes loop (numpy arrays prepared once), and
the caller's liblbfgs fit (tests/lbfgs_fit_child.py) on the same library.
    [TRPO_LIB=lib.so] python tools/baseline_eval_timing.py [reps]"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import numpy as np  # noqa: E402
import trpo_amd  # noqa: E402
from trpo_amd import synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    L = [16, 16, 16, 1]
    x, obs, tgt = synth.make_baseline_problem(L, 20, 150)
    lib = trpo_amd.lib()
    with trpo_amd.Baseline(L, "lttl", device=0) as b:
        b.set_data(obs, tgt, 20, 150)
        x = np.ascontiguousarray(x, np.float64)
        g = np.zeros(x.size)
        f0, g0 = b.evaluate(x)
        fn = lib.trpo_baseline_evaluate
        t = np.zeros(reps)
        for r in range(reps):
            t0 = time.perf_counter()
            fn(b._h, x, g, x.size, None)
            t[r] = time.perf_counter() - t0
        assert np.array_equal(g, g0), "evaluate not repeatable"
    t = np.sort(t) * 1e6
    print("evaluate host-visible us: p10 %.2f med %.2f p90 %.2f (%d calls, %s)" % (
        t[reps // 10], t[reps // 2], t[reps * 9 // 10], reps, os.path.basename(trpo_amd.LIB_PATH)), flush=True)
    child = os.path.join(ROOT, "tests", "lbfgs_fit_child.py")
    if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_lbfgs.so")):
        p = subprocess.run([sys.executable, child, "9"], capture_output=True, text=True, timeout=170)
        print("liblbfgs fit:", p.stdout.strip().splitlines()[-1] if p.returncode == 0 else p.stderr[-500:], flush=True)


if __name__ == "__main__":
    main()
