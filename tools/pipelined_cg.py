"""CPU study: standard CG (src/TRPO_CG.c) vs the pipelined (Ghysels-Vanroose) recurrence on the
golden CG cases, with the fp64 oracle FVP and with an fp32-per-sample emulated FVP (numpy).
Both use exactly maxiter FVPs; the pipelined form takes its dot products off the FVP's critical
path.  Prints relative L2 of the step vs the reference golden and the rdotr histories."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, p) for p in ("oracle", "tests", "trpo-robot-control_amd")]
import numpy as np, oracle, cases


def fvp32(L, th, obs, std, v, lam):
    """fp32 per-sample math, fp64 sums (the device fp32 contract)."""
    def unpack(t, dt):
        W, B, pos = [], [], 0
        for i in range(3):
            W.append(t[pos:pos + L[i] * L[i + 1]].reshape(L[i], L[i + 1]).astype(dt)); pos += L[i] * L[i + 1]
            B.append(t[pos:pos + L[i + 1]].astype(dt)); pos += L[i + 1]
        return W, B
    dt = np.float32
    W, B = unpack(th, dt); VW, VB = unpack(v, dt); x = obs.astype(dt); iv = (1.0 / std ** 2).astype(dt)
    y1 = np.tanh(x @ W[0] + B[0]); ry1 = (x @ VW[0] + VB[0]) * (1 - y1 * y1)
    y2 = np.tanh(y1 @ W[1] + B[1]); ry2 = (ry1 @ W[1] + y1 @ VW[1] + VB[1]) * (1 - y2 * y2)
    g3 = (ry2 @ W[2] + y2 @ VW[2] + VB[2]) * iv
    g2 = (g3 @ W[2].T) * (1 - y2 * y2); g1 = (g2 @ W[1].T) * (1 - y1 * y1)
    parts = []
    for a, g in ((x, g1), (y1, g2), (y2, g3)):
        parts += [(a.astype(np.float64).T @ g.astype(np.float64)).ravel(), g.astype(np.float64).sum(0)]
    n = obs.shape[0]
    r = np.concatenate(parts) / n
    return np.concatenate([r, 2 * v[-L[-1]:]]) + lam * v


def cg_std(fv, b, M, th):
    x = np.zeros_like(b); r = b.copy(); p = b.copy(); rr = r @ r; hist = [rr]
    for it in range(M):
        if rr < th: break
        z = fv(p); a = rr / (p @ z); x += a * p; r -= a * z; nr = r @ r; p = r + nr / rr * p; rr = nr; hist.append(rr)
    return x, hist


def cg_pipe(fv, b, M, th):
    x = np.zeros_like(b); r = b.copy(); w = fv(r)
    z = s = p = np.zeros_like(b); gam_prev = alpha_prev = None; hist = []
    for i in range(M):
        gam = r @ r; delta = w @ r; hist.append(gam)
        if gam < th: break
        q = fv(w) if i < M - 1 else np.zeros_like(b)     # the last q is never used
        if i == 0: beta, alpha = 0.0, gam / delta
        else:
            beta = gam / gam_prev; alpha = gam / (delta - beta * gam / alpha_prev)
        z = q + beta * z; s = w + beta * s; p = r + beta * p
        x = x + alpha * p; r = r - alpha * s; w = w - alpha * z
        gam_prev, alpha_prev = gam, alpha
    else:
        hist.append(r @ r)
    return x, hist


names = sys.argv[1:] or [c["name"] for c in cases.manifest() if c["kind"] == "cg"]
for name in names:
    c = cases.case(name); X = cases.inputs(c); exp = cases.expected(c)
    L, th, obs, std, lam = X["layers"], X["theta"], X["obs"], X["std"], X["damping"]
    f64 = lambda v: oracle.fvp(L, X["acfunc"], th, obs, std, v, lam)[0]
    f32 = lambda v: fvp32(L, th, obs, std, v, lam)
    out = [name]
    for tag, fv in (("fp64", f64), ("fp32", f32)):
        xs, hs = cg_std(fv, X["vin"], c["maxiter"], c["resth"])
        xp, hp = cg_pipe(fv, X["vin"], c["maxiter"], c["resth"])
        out.append("%s std %.2e pipe %.2e (iters %d/%d)" % (tag, cases.rel_l2(xs, exp), cases.rel_l2(xp, exp), len(hs) - 1, len(hp) - 1))
    print(" | ".join(out), flush=True)
