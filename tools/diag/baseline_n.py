"""Baseline evaluate at several sample counts (for a kernel trace: is baseline_kernel per-wave latency?).
usage: python tools/diag/baseline_n.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import trpo_amd  # noqa: E402
from trpo_amd import synth  # noqa: E402

L = [16, 16, 16, 1]
for nep, eplen in ((1, 64), (4, 160), (20, 150), (80, 150)):
    x, obs, tgt = synth.make_baseline_problem(L, nep, eplen)
    with trpo_amd.Baseline(L, "lttl") as b:
        b.set_data(obs, tgt, nep, eplen)
        for _ in range(5):
            b.evaluate(x)
        t0 = time.perf_counter()
        for _ in range(50):
            b.evaluate(x)
        print("N=%d evaluate %.1f us host-visible" % (nep * eplen, 1e6 * (time.perf_counter() - t0) / 50), flush=True)
