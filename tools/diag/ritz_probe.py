"""CPU: can a Ritz-value test on the CG coefficients predict where the reference's fp64 CG loses
orthogonality (Paige: |q_i . r_k| ~ eps ||A|| / (Ritz residual of pair i))?  For each case, the
reference's recurrence in numpy fp64 on the oracle FVP: alpha_k, beta_k -> Lanczos T_k -> Ritz values and
residual bounds beta_k |s_k,i|; printed: the smallest relative Ritz residual over the steps, the step
error of the reorthogonalised recurrence against the plain one (the quantity the fp32 path gets wrong)."""
import os
import sys

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import numpy as np  # noqa: E402

import cases  # noqa: E402
import oracle  # noqa: E402
from trpo_amd import synth  # noqa: E402


def cg(F, b, maxiter, resth, reorth):
    x = np.zeros_like(b)
    r, p = b.copy(), b.copy()
    rr = r @ r
    al, be, Q = [], [], []
    for k in range(maxiter):
        if rr < resth:
            break
        z = F(p)
        a = rr / (p @ z)
        x += a * p
        r = r - a * z
        if reorth:
            for q in Q:
                r = r - (q @ r) * q
        Q.append(r / np.linalg.norm(r))
        nr = r @ r
        al.append(a)
        be.append(nr / rr)
        p = r + nr / rr * p
        rr = nr
    return x, np.array(al), np.array(be)


def ritz_min(al, be):
    """smallest relative Ritz residual over k (Lanczos T_k from CG coefficients)."""
    best = np.inf
    for k in range(1, len(al) + 1):
        T = np.zeros((k, k))
        for j in range(k):
            T[j, j] = 1.0 / al[j] + (be[j - 1] / al[j - 1] if j > 0 else 0.0)
            if j + 1 < k:
                T[j, j + 1] = T[j + 1, j] = np.sqrt(be[j]) / al[j]
        w, S = np.linalg.eigh(T)
        bk = np.sqrt(be[k - 1]) / al[k - 1]          # T_{k+1,k}
        res = bk * np.abs(S[-1, :]) / np.max(np.abs(w))
        best = min(best, float(res.min()))
    return best


def report(name, layers, acts, th, obs, std, b, maxiter=10, resth=1e-10, damping=0.1):
    F = lambda p: oracle.fvp(layers, acts, th, obs, std, p, damping)[0]  # noqa: E731
    xp, al, be = cg(F, b, maxiter, resth, False)
    xr, _, _ = cg(F, b, maxiter, resth, True)
    print("%-40s min rel Ritz residual %.2e   |reorth - plain| %.2e" % (name, ritz_min(al, be),
                                                                       np.linalg.norm(xr - xp) / np.linalg.norm(xp)),
          flush=True)


def noisy_probe():
    """the same Ritz test from coefficients carrying the fp32 path's ~1e-7 relative noise"""
    rng = np.random.default_rng(0)
    print("--- coefficients perturbed by 1e-7 relative (the fp32 trajectory's accuracy)")
    for seed in (23, 11, 20, 25, 21, 31, 12):
        layers, acts, n, std = _draw(seed)
        th = synth.make_theta(layers, seed=100 + seed)
        obs = synth.make_obs(n, layers[0], seed=200 + seed)
        mean, action, adv = synth.make_rollout(layers, acts, th, obs, std, seed=500 + seed)
        b, _ = oracle.policy_grad(layers, acts, th, obs, mean, action, adv)
        F = lambda p: oracle.fvp(layers, acts, th, obs, std, p, 0.1)[0]  # noqa: E731
        _, al, be = cg(F, b, 10, 1e-10, True)
        vals = [ritz_min(al * (1 + 1e-7 * rng.standard_normal(al.size)), be * (1 + 1e-7 * rng.standard_normal(be.size)))
                for _ in range(5)]
        print("draw %d: reorth coefficients %.2e, noisy %s" % (seed, ritz_min(al, be), " ".join("%.1e" % v for v in vals)))



if __name__ == "__main__":
    for name in ("fix_cg_n3150_th1e-10", "fix_cg_n3150_th0", "syn_sigma_cg", "syn_arm_cg_n50000"):
        c = cases.case(name)
        X = cases.inputs(c)
        report(name, X["layers"], X["acfunc"], X["theta"], X["obs"], X["std"], X["vin"], c["maxiter"], c["resth"],
               X["damping"])
    from test_gpu_random_shapes import _draw  # noqa: E402

    for seed in range(36):
        layers, acts, n, std = _draw(seed)
        th = synth.make_theta(layers, seed=100 + seed)
        obs = synth.make_obs(n, layers[0], seed=200 + seed)
        mean, action, adv = synth.make_rollout(layers, acts, th, obs, std, seed=500 + seed)
        b, _ = oracle.policy_grad(layers, acts, th, obs, mean, action, adv)
        report("draw %d %s %s" % (seed, layers, acts), layers, acts, th, obs, std, b)


    noisy_probe()
