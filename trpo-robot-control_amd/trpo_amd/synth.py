"""Seeded synthetic TRPO inputs, bit-identical on every host.

The generator uses only integer arithmetic (splitmix64) and exact fp64
operations -- no transcendental functions -- so the CPU oracle, the reference
build and the MI355X path all see bit-identical inputs, here and on the GPU box.

Distributions:
  * observations ~ U[-0.17, 0.19]    (the ArmTestData.txt range)
  * W ~ N(0, 1/fan_in)   via Irwin-Hall(12) - 6, b = 0, logstd = 0
  * v ~ U[0, 1)          (as ArmTestFVP.txt column 1)
  * CG right-hand side b ~ N(0, 1e-2^2)
  * TRPO_Update rollouts: Mean = the policy's own output on the observations,
    Action = Mean + Std * N(0, 1), Advantage ~ N(0, 1).  The policy mean uses
    tanh through Lambert's continued fraction (exact IEEE +,-,*,/ only), so it
    is still bit-identical on every host.
"""
from __future__ import annotations

import numpy as np

SEED = 20261015
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# stream ids keep the different inputs independent
STREAM_OBS, STREAM_W, STREAM_V, STREAM_B, STREAM_ACT, STREAM_ADV, STREAM_RET = 1, 2, 3, 4, 5, 6, 7


def _splitmix(seed: int, stream: int, count: int, offset: int = 0) -> np.ndarray:
    base = np.uint64((seed * 0x100000001B3 + stream * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        i = np.arange(offset + 1, offset + count + 1, dtype=np.uint64)
        z = base + i * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, stream: int, count: int, lo: float = 0.0, hi: float = 1.0,
            offset: int = 0) -> np.ndarray:
    u = (_splitmix(seed, stream, count, offset) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return lo + (hi - lo) * u


def normal(seed: int, stream: int, count: int, sigma: float = 1.0) -> np.ndarray:
    """Irwin-Hall(12) approximation of N(0, sigma^2): exact arithmetic only."""
    u = uniform(seed, stream, 12 * count).reshape(count, 12)
    acc = np.zeros(count)
    for j in range(12):          # fixed summation order
        acc = acc + u[:, j]
    return (acc - 6.0) * sigma


def num_params(layers) -> int:
    """src/TRPO_Util.c:7-17."""
    p = 0
    for i in range(len(layers) - 1):
        p += layers[i] * layers[i + 1] + layers[i + 1]
    return p + layers[-1]


def make_theta(layers, seed: int = SEED, logstd: float = 0.0) -> np.ndarray:
    """Flat parameters in the reference layout: W[i] [in][out], B[i], ..., LogStd."""
    parts = []
    for i in range(len(layers) - 1):
        fan_in, out = layers[i], layers[i + 1]
        w = normal(seed + 1000 * i, STREAM_W, fan_in * out, sigma=1.0 / np.sqrt(float(fan_in)))
        parts += [w, np.zeros(out)]
    parts.append(np.full(layers[-1], logstd))
    return np.concatenate(parts)


def make_obs(n: int, obs_dim: int, seed: int = SEED, start: int = 0) -> np.ndarray:
    """Rows [start, start + n) of the seeded observation stream (a rank generates only its shard)."""
    return uniform(seed, STREAM_OBS, n * obs_dim, -0.17, 0.19, offset=start * obs_dim).reshape(n, obs_dim)


def make_v(P: int, seed: int = SEED) -> np.ndarray:
    return uniform(seed, STREAM_V, P)


def make_b(P: int, seed: int = SEED) -> np.ndarray:
    return normal(seed, STREAM_B, P, sigma=1e-2)


def tanh_cf(x: np.ndarray, depth: int = 24) -> np.ndarray:
    """tanh via Lambert's continued fraction x / (1 + x^2 / (3 + x^2 / (5 + ...))),
    exact arithmetic only; agrees with libm tanh to ~1 ulp for |x| < 4."""
    x = np.asarray(x, dtype=np.float64)
    x2 = x * x
    t = np.full_like(x, 2.0 * depth + 1.0)
    for k in range(depth, 0, -1):
        t = (2.0 * k - 1.0) + x2 / t
    return x / t


def policy_mean(layers, acfunc: str, theta: np.ndarray, obs: np.ndarray) -> np.ndarray:
    """Forward pass of the policy MLP (src/TRPO_Update.c:262-293), fixed-order sums,
    no BLAS, so the result does not depend on the host."""
    y = np.asarray(obs, dtype=np.float64)
    pos = 0
    for i in range(len(layers) - 1):
        fin, out = layers[i], layers[i + 1]
        W = theta[pos:pos + fin * out].reshape(fin, out)
        B = theta[pos + fin * out:pos + fin * out + out]
        pos += fin * out + out
        x = np.broadcast_to(B, (y.shape[0], out)).copy()
        for k in range(fin):
            x = x + y[:, k:k + 1] * W[k:k + 1, :]
        a = acfunc[i + 1]
        if a == "t":
            x = tanh_cf(x)
        elif a == "o":
            x = 0.1 * x
        elif a == "s":
            x = 0.5 + 0.5 * tanh_cf(0.5 * x)
        y = x
    return y


def make_rollout(layers, acfunc: str, theta: np.ndarray, obs: np.ndarray, std, seed: int = SEED):
    """(mean [n][A], action [n][A], advantage [n]) for a TRPO_Update data file."""
    n, A = obs.shape[0], layers[-1]
    mean = policy_mean(layers, acfunc, theta, obs)
    action = mean + np.asarray(std, dtype=np.float64) * normal(seed, STREAM_ACT, n * A).reshape(n, A)
    adv = normal(seed, STREAM_ADV, n)
    return mean, action, adv


def make_baseline_problem(layers_base, num_ep: int, ep_len: int, seed: int = SEED, scale: float = 1.0,
                          pad_value: float = 0.0):
    """Value-baseline fit inputs (src/TRPO_Baseline.c): x [PaddedParams] (the baseline MLP's
    weights and biases, zero-/pad_value-padded to a multiple of 16), observations
    [num_ep * ep_len][layers_base[0] - 1] and regression targets (returns ~ N(0, 2^2))."""
    npar = num_params(layers_base) - layers_base[-1]
    padded = (npar + 15) // 16 * 16
    x = np.full(padded, pad_value)
    x[:npar] = scale * make_theta(layers_base, seed)[:npar]
    n = num_ep * ep_len
    obs = make_obs(n, layers_base[0] - 1, seed)
    target = normal(seed, STREAM_RET, n, sigma=2.0)
    return x, obs, target


def write_model_file(path: str, theta: np.ndarray) -> None:
    """One value per line (src/TRPO_FVP.c:670-699)."""
    with open(path, "w") as f:
        f.write("\n".join("%.17g" % x for x in theta))
        f.write("\n")


def write_data_file(path: str, obs: np.ndarray, std: np.ndarray, mean: np.ndarray | None = None,
                    action: np.ndarray | None = None, adv: np.ndarray | None = None) -> None:
    """Per sample: Mean[A] Std[A] Obs[O] Action[A] Adv (src/TRPO_FVP.c:731-762).
    Missing Mean / Action / Advantage columns are written as zeros (the FVP/CG path
    never reads them; TRPO_Update does)."""
    n, _ = obs.shape
    A = len(std)
    mean = np.zeros((n, A)) if mean is None else mean
    action = np.zeros((n, A)) if action is None else action
    adv = np.zeros(n) if adv is None else adv
    table = np.concatenate([mean, np.broadcast_to(std, (n, A)), obs, action, adv[:, None]], axis=1)
    np.savetxt(path, table, fmt="%.17g")


def write_vector_file(path: str, v: np.ndarray) -> None:
    np.savetxt(path, np.asarray(v, dtype=np.float64), fmt="%.17g")
