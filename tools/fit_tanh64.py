"""Coefficients of the fp64 tanh used by the device fp64 paths (trpo_update.hip tanh64):
|x| < 0.55: tanh(x) = x + x^3 Q(x^2), Q a degree-N polynomial fitted in extended precision
(np.longdouble, x86 80-bit) by least squares on Chebyshev nodes; |x| >= 0.55: 1 - 2 / (e^{2|x|} + 1).
Prints the coefficients and the max relative error of the fp64-evaluated polynomial vs tanhl."""
import numpy as np
ld = np.longdouble
T = ld("0.55")
N = int(__import__("sys").argv[1]) if len(__import__("sys").argv) > 1 else 9
k = np.arange(4000, dtype=ld)
u = (T * T) * (ld(1) - np.cos((k + ld(0.5)) * ld(np.pi) / ld(4000))) / ld(2)   # Chebyshev nodes on [0, T^2]
u = u[u > ld(1e-30)]
x = np.sqrt(u)
f = (np.tanh(x) - x) / (x * u)                       # target Q(u)
V = np.vander(u, N + 1, increasing=True)
w = ld(1) / np.abs(f)                                 # relative weighting
c = np.linalg.lstsq((V * w[:, None]).astype(np.float64), (f * w).astype(np.float64), rcond=None)[0]
# refine in long double with one Newton-style correction of the residual
c = c.astype(ld)
for _ in range(3):
    r = (f - V @ c) * w
    dc = np.linalg.lstsq((V * w[:, None]).astype(np.float64), r.astype(np.float64), rcond=None)[0]
    c = c + dc.astype(ld)
cd = c.astype(np.float64)
xs = np.linspace(1e-6, 0.55, 200001)
def poly(x):
    u = x * x
    q = np.zeros_like(x) + cd[N]
    for i in range(N - 1, -1, -1):
        q = q * u + cd[i]
    return x + (x * u) * q
ref = np.tanh(xs.astype(ld))
err = np.max(np.abs((poly(xs).astype(ld) - ref) / ref))
e2 = np.linspace(0.55, 25, 200001)
t2 = 1.0 - 2.0 / (np.exp(2 * e2) + 1.0)
err2 = np.max(np.abs((t2.astype(ld) - np.tanh(e2.astype(ld))) / np.tanh(e2.astype(ld))))
print("degree", N, "max rel err poly %.3e  exp-branch %.3e" % (err, err2))
print(", ".join("%.17e" % v for v in cd))
