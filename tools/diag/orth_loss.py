"""CPU emulation: how far from orthogonal does each new CG residual come out BEFORE the
reorthogonalisation, in the fp32-FVP trajectory the device runs -- per golden and for random draw 23?
F p is the oracle's fp64 FVP plus a direction-dependent perturbation of relative size eps (the fp32
FVP's rounding); the CG is the device's reorthogonalised fp64 recurrence.  Printed per case:
max over steps of sum(c^2) / |r'|^2 (the statistic the device's block reduction already forms), the
step's rel-L2 from the reference's plain fp64 CG, and the reference's own loss of orthogonality
(max |q_i . r_k| / |r_k| in ITS trajectory)."""
import os
import sys

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import numpy as np  # noqa: E402

import cases  # noqa: E402
import oracle  # noqa: E402
from trpo_amd import synth  # noqa: E402


def make_F(layers, acts, th, obs, std, damping, eps):
    def F(p):
        z, _ = oracle.fvp(layers, acts, th, obs, std, p, damping)
        if eps:
            h = np.frombuffer(np.ascontiguousarray(p, np.float64).tobytes(), np.uint64)
            rng = np.random.default_rng(int(h.sum() % (2 ** 63)))
            z = z + eps * np.linalg.norm(z) / np.sqrt(z.size) * rng.standard_normal(z.size)
        return z
    return F


def cg(F, b, maxiter, resth, reorth):
    x = np.zeros_like(b)
    r, p = b.copy(), b.copy()
    rr = r @ r
    Q, worst, ref_loss = [], 0.0, 0.0
    for k in range(maxiter):
        if rr < resth:
            break
        z = F(p)
        a = rr / (p @ z)
        x += a * p
        r = r - a * z
        if Q:
            c = np.array([q @ r for q in Q])
            worst = max(worst, float(c @ c / (r @ r)))
            ref_loss = max(ref_loss, float(np.max(np.abs(c)) / np.linalg.norm(r)))
            if reorth:
                for q, ci in zip(Q, c):
                    r = r - ci * q
        Q.append(r / np.linalg.norm(r) if False else None)
        Q[-1] = (r / np.linalg.norm(r))
        nr = r @ r
        p = r + nr / rr * p
        rr = nr
    return x, worst, ref_loss


def report(name, layers, acts, th, obs, std, b, maxiter, resth, damping=0.1):
    F64 = make_F(layers, acts, th, obs, std, damping, 0.0)
    xr, _, loss_ref = cg(F64, b, maxiter, resth, reorth=False)
    F32 = make_F(layers, acts, th, obs, std, damping, 1e-7)
    xd, worst, _ = cg(F32, b, maxiter, resth, reorth=True)
    print("%-28s max sum(c^2)/|r'|^2 = %.2e   step vs ref %.2e   ref's own orth. loss %.2e"
          % (name, worst, np.linalg.norm(xd - xr) / np.linalg.norm(xr), loss_ref), flush=True)


for name in ("fix_cg_n3150_th1e-10", "fix_cg_n3150_th0", "fix_cg_n2400_th1e-10", "syn_sigma_cg", "syn_arm_cg_n50000"):
    c = cases.case(name)
    X = cases.inputs(c)
    report(name, X["layers"], X["acfunc"], X["theta"], X["obs"], X["std"], X["vin"], c["maxiter"], c["resth"],
           X["damping"])
for name in ("fix_update_n3150", "syn_update_sigma_n5000", "syn_update_arm_n20000"):
    c = cases.case(name)
    X = cases.update_inputs(c)
    b, _ = oracle.policy_grad(X["layers"], X["acfunc"], X["theta"], X["obs"], X["mean"], X["action"], X["adv"])
    report(name, X["layers"], X["acfunc"], X["theta"], X["obs"], X["std"], b, 10, 1e-10, X["damping"])
from test_gpu_random_shapes import _draw  # noqa: E402

for seed in [int(s) for s in sys.argv[1:]] or [23, 0, 1, 2, 5, 8, 11, 14, 17, 20, 26, 29, 32, 35]:
    layers, acts, n, std = _draw(seed)
    th = synth.make_theta(layers, seed=100 + seed)
    obs = synth.make_obs(n, layers[0], seed=200 + seed)
    mean, action, adv = synth.make_rollout(layers, acts, th, obs, std, seed=500 + seed)
    b, _ = oracle.policy_grad(layers, acts, th, obs, mean, action, adv)
    report("draw %d %s %s" % (seed, layers, acts), layers, acts, th, obs, std, b, 10, 1e-10)
