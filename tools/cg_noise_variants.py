"""numpy emulation: which CG formulation reproduces the reference's fp64 10-iteration CG step when
the FVP carries fp32 rounding noise that depends on the direction p?  CPU only.

The fp32 device FVP is F p + delta(p), |delta| ~ 1e-7 |F p|, with delta a NON-linear function of p
(rounding of p and of the p-dependent R chains).  tools/precision_emulation.py showed plain CG
amplifies that to 8e-4 on the 2x64 update case.  Variants:
  plain     the reference recurrence (src/TRPO_CG.c:45-104)
  reorth    plain + Gram-Schmidt of each new residual against the previous ones (fp64)
  split     FVP of p = p_hi + p_lo (two fp32 FVPs summed in fp64)
  fp64      the fp64 FVP (the precision mode)
Usage: python tools/cg_noise_variants.py [case ...]
"""
import sys

sys.path[:0] = ['oracle', 'tests', 'trpo-robot-control_amd']
import numpy as np  # noqa: E402

import cases  # noqa: E402
import oracle  # noqa: E402


def unpack(t, L, dt):
    Ws, Bs, pos = [], [], 0
    for i in range(3):
        W = t[pos:pos + L[i] * L[i + 1]].reshape(L[i], L[i + 1]).astype(dt)
        pos += L[i] * L[i + 1]
        B = t[pos:pos + L[i + 1]].astype(dt)
        pos += L[i + 1]
        Ws.append(W)
        Bs.append(B)
    return Ws, Bs


def tanh_ref(x):
    return np.tanh(x)


class Emu:
    """FVP of a 3-weight-layer tanh policy (acfunc 'lttl'); dt = per-sample arithmetic type."""

    def __init__(self, L, th, obs, std, damping):
        self.L, self.n, self.std, self.damping = L, obs.shape[0], std, damping
        self.th, self.obs = th, obs
        self.cache = {}

    def fwd(self, dt):
        if dt not in self.cache:
            W, B = unpack(self.th, self.L, dt)
            x = self.obs.astype(dt)
            y1 = np.tanh(x @ W[0] + B[0])
            y2 = np.tanh(y1 @ W[1] + B[1])
            self.cache[dt] = (W, x, y1, y2)
        return self.cache[dt]

    def fvp(self, v, dt=np.float32, rdt=None):
        """dt: forward (y, W) type; rdt: type of the p-dependent chains (default dt)"""
        rdt = rdt or dt
        L, n = self.L, self.n
        W, x, y1, y2 = self.fwd(dt)
        W = [w.astype(rdt) for w in W]
        x, y1, y2 = x.astype(rdt), y1.astype(rdt), y2.astype(rdt)
        VW, VB = unpack(v, L, rdt)
        rx1 = x @ VW[0] + VB[0]
        ry1 = rx1 * (1 - y1 * y1)
        rx2 = ry1 @ W[1] + y1 @ VW[1] + VB[1]
        ry2 = rx2 * (1 - y2 * y2)
        rx3 = ry2 @ W[2] + y2 @ VW[2] + VB[2]
        g3 = rx3 / (self.std.astype(rdt) ** 2)
        g2 = (g3 @ W[2].T) * (1 - y2 * y2)
        g1 = (g2 @ W[1].T) * (1 - y1 * y1)
        res = []
        for a, g in [(x, g1), (y1, g2), (y2, g3)]:
            acc = np.zeros((a.shape[1], g.shape[1]), np.float64)
            for s in range(0, n, 256):
                acc += (a[s:s + 256].T @ g[s:s + 256]).astype(np.float64)
            res.append(acc.ravel())
            res.append(g.sum(0, dtype=np.float64))
        r = np.concatenate(res) / n
        A = L[-1]
        return np.concatenate([r, 2 * v[-A:]]) + self.damping * v


def cg(fv, b, iters=10, th=1e-10, reorth=False):
    x = np.zeros_like(b)
    r = b.copy()
    p = b.copy()
    rr = r @ r
    R = [r / np.sqrt(rr)]
    for it in range(iters):
        if rr < th:
            break
        z = fv(p)
        a = rr / (p @ z)
        x += a * p
        r = r - a * z
        if reorth:
            for q in R:
                r = r - (q @ r) * q
        nr = r @ r
        R.append(r / np.sqrt(nr))
        p = r + nr / rr * p
        rr = nr
    return x


def run(name):
    c = cases.case(name)
    if c['kind'] == 'update':
        X = cases.update_inputs(c)
        b, _ = oracle.policy_grad(X['layers'], X['acfunc'], X['theta'], X['obs'], X['mean'], X['action'], X['adv'])
        ref = oracle.update(X['layers'], X['acfunc'], X['theta'], X['obs'], X['mean'], X['action'], X['adv'],
                            X['std'])['x']
        maxit, th = 10, 1e-10
    else:
        X = cases.inputs(c)
        b = X['vin']
        ref = cases.expected(c)
        maxit, th = c['maxiter'], c['resth']
    if X['acfunc'] != 'lttl' or len(X['layers']) != 4:
        print(name, 'skipped (emulation covers lttl 3-layer only)')
        return
    e = Emu(X['layers'], X['theta'], X['obs'], X['std'], X['damping'])
    f32 = lambda a: a.astype(np.float32).astype(np.float64)
    variants = {
        'plain fp32': lambda: cg(lambda p: e.fvp(p), b, maxit, th),
        'reorth fp32': lambda: cg(lambda p: e.fvp(p), b, maxit, th, reorth=True),
        'split p fp32': lambda: cg(lambda p: e.fvp(f32(p)) + e.fvp(p - f32(p)), b, maxit, th),
        'fwd32 r64': lambda: cg(lambda p: e.fvp(p, np.float32, np.float64), b, maxit, th),
        'fp64': lambda: cg(lambda p: e.fvp(p, np.float64), b, maxit, th),
    }
    for k, f in variants.items():
        x = f()
        print('%-22s %-14s relL2 %.3e' % (name, k, np.linalg.norm(x - ref) / np.linalg.norm(ref)), flush=True)


if __name__ == '__main__':
    for nm in sys.argv[1:] or ['syn_update_2x64_n8192']:
        run(nm)
