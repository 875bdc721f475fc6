import sys, os
sys.path[:0] = [os.path.join(os.getcwd(), "trpo-robot-control_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np
import trpo_amd
from trpo_amd import synth
import test_gpu_large_n as t
for L, n in t.CASES:
    P = synth.num_params(L); A = L[-1]; nw = P - A
    u = np.random.default_rng(23).standard_normal(P)
    with t._ctx(n, layers=L) as c:
        zu = c.fvp(u); kn = c.kernel_name
    n1 = n // 2 + 37
    with t._ctx(n1, layers=L) as c1: z1 = c1.fvp(u)
    with t._ctx(n - n1, start=n1, layers=L) as c2: z2 = c2.fvp(u)
    full = (zu[:nw] - t.LAM * u[:nw]) * n
    parts = (z1[:nw] - t.LAM * u[:nw]) * n1 + (z2[:nw] - t.LAM * u[:nw]) * (n - n1)
    print(L, n, kn, "decomposition relL2", t._rel(full, parts), flush=True)
