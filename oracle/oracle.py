"""ctypes view of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The checker for the MI355X path (and bench.py's "port" CPU baseline).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# TRPO_ORACLE_LIB: another build of the same restatement (tests/test_asan.py: the ASan + UBSan one)
LIB_PATH = os.environ.get("TRPO_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
REF_DRIVER = os.path.join(HERE, "_ref", "ref_driver")
REF_DRIVER_FAST = os.path.join(HERE, "_ref", "ref_driver_fast")

_lib = None
_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_sp = np.ctypeslib.ndpointer(dtype=np.uintp, flags="C_CONTIGUOUS")


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_num_params.restype = C.c_size_t
        L.oracle_num_params.argtypes = [_sp, C.c_size_t]
        L.oracle_fvp.restype = C.c_double
        L.oracle_fvp.argtypes = [C.c_size_t, _sp, C.c_char_p, _dp, _dp, C.c_size_t, _dp, C.c_double, _dp,
                                 _dp, C.c_int]
        L.oracle_cg.restype = C.c_double
        L.oracle_cg.argtypes = [C.c_size_t, _sp, C.c_char_p, _dp, _dp, C.c_size_t, _dp, C.c_double, _dp,
                                C.c_size_t, C.c_double, _dp, _dp, _dp, C.POINTER(C.c_size_t), C.c_int, C.c_int]
        L.oracle_load_model.restype = C.c_int
        L.oracle_load_model.argtypes = [C.c_char_p, C.c_size_t, _sp, _dp]
        L.oracle_load_data.restype = C.c_int
        L.oracle_load_data.argtypes = [C.c_char_p, C.c_size_t, _sp, C.c_size_t, _dp, _dp, C.c_void_p]
        L.oracle_forward.restype = C.c_int
        L.oracle_forward.argtypes = [C.c_size_t, _sp, C.c_char_p, _dp, _dp, C.c_size_t, _dp]
        L.oracle_policy_grad.restype = C.c_int
        L.oracle_policy_grad.argtypes = [C.c_size_t, _sp, C.c_char_p, _dp, _dp, _dp, _dp, _dp, C.c_size_t, C.c_int,
                                         _dp, C.POINTER(C.c_double)]
        L.oracle_surrogate_sum.restype = C.c_double
        L.oracle_surrogate_sum.argtypes = [C.c_size_t, _sp, C.c_char_p, _dp, _dp, _dp, _dp, _dp, _dp, C.c_size_t]
        L.oracle_update.restype = C.c_double
        L.oracle_update.argtypes = [C.c_size_t, _sp, C.c_char_p, _dp, _dp, _dp, _dp, _dp, _dp, C.c_size_t,
                                    C.c_double, C.c_size_t, C.c_double, C.c_double, C.c_int, C.c_double,
                                    _dp, _dp, _dp, _dp, _dp, C.POINTER(C.c_int), C.c_int]
        L.oracle_baseline_evaluate.restype = C.c_double
        L.oracle_baseline_evaluate.argtypes = [C.c_size_t, _sp, C.c_char_p, _dp, C.c_int, _dp, _dp, C.c_size_t,
                                               C.c_size_t, _dp, _dp]
        L.oracle_load_rollout.restype = C.c_int
        L.oracle_load_rollout.argtypes = [C.c_char_p, C.c_size_t, _sp, C.c_size_t, _dp, _dp, _dp, _dp, _dp]
        _lib = L
    return _lib


def _ls(layers):
    return np.ascontiguousarray(layers, dtype=np.uintp)


def num_params(layers) -> int:
    return int(lib().oracle_num_params(_ls(layers), len(layers)))


def fvp(layers, acfunc, theta, obs, std, v, damping=0.1, threads=1):
    """Returns (Fv, compute_seconds)."""
    obs = np.ascontiguousarray(obs, dtype=np.float64)
    out = np.zeros(num_params(layers))
    t = lib().oracle_fvp(len(layers), _ls(layers), acfunc.encode(), np.ascontiguousarray(theta, np.float64),
                         obs, obs.shape[0], np.ascontiguousarray(std, np.float64), damping,
                         np.ascontiguousarray(v, np.float64), out, threads)
    if t < 0:
        raise RuntimeError("oracle_fvp failed")
    return out, t


def cg(layers, acfunc, theta, obs, std, b, maxiter=10, resth=1e-10, damping=0.1, threads=1, verbose=False):
    """Returns dict(x, rdotr, xnorm, iters, seconds)."""
    obs = np.ascontiguousarray(obs, dtype=np.float64)
    P = num_params(layers)
    x = np.zeros(P)
    rh = np.zeros(maxiter + 1)
    xh = np.zeros(maxiter + 1)
    it = C.c_size_t(0)
    t = lib().oracle_cg(len(layers), _ls(layers), acfunc.encode(), np.ascontiguousarray(theta, np.float64), obs,
                        obs.shape[0], np.ascontiguousarray(std, np.float64), damping,
                        np.ascontiguousarray(b, np.float64), maxiter, resth, x, rh, xh, C.byref(it), threads,
                        1 if verbose else 0)
    if t < 0:
        raise RuntimeError("oracle_cg failed")
    n = it.value + 1
    return dict(x=x, rdotr=rh[:n], xnorm=xh[:n], iters=it.value, seconds=t)


def load_model(path, layers):
    th = np.zeros(num_params(layers))
    if lib().oracle_load_model(path.encode(), len(layers), _ls(layers), th):
        raise IOError(path)
    return th


def load_data(path, layers, n):
    obs = np.zeros((n, layers[0]))
    std = np.zeros(layers[-1])
    if lib().oracle_load_data(path.encode(), len(layers), _ls(layers), n, obs, std, None):
        raise IOError(path)
    return obs, std


def forward(layers, acfunc, theta, obs):
    obs = np.ascontiguousarray(obs, dtype=np.float64)
    out = np.zeros((obs.shape[0], layers[-1]))
    lib().oracle_forward(len(layers), _ls(layers), acfunc.encode(), np.ascontiguousarray(theta, np.float64), obs,
                         obs.shape[0], out)
    return out


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def policy_grad(layers, acfunc, theta, obs, mean, action, adv, normalise=True):
    """src/TRPO_Update.c:254-378.  Returns (b, sum(adv))."""
    obs = _f64(obs)
    b = np.zeros(num_params(layers))
    s = C.c_double(0.0)
    lib().oracle_policy_grad(len(layers), _ls(layers), acfunc.encode(), _f64(theta), obs, _f64(mean), _f64(action),
                             _f64(adv), obs.shape[0], 1 if normalise else 0, b, C.byref(s))
    return b, s.value


def surrogate_sum(layers, acfunc, theta_new, obs, mean, action, adv, std):
    """sum_n Adv_n exp(LLD_n) (src/TRPO_Update.c:951-981)."""
    obs = _f64(obs)
    return lib().oracle_surrogate_sum(len(layers), _ls(layers), acfunc.encode(), _f64(theta_new), obs, _f64(mean),
                                      _f64(action), _f64(adv), _f64(std), obs.shape[0])


def update(layers, acfunc, theta, obs, mean, action, adv, std, damping=0.1, maxiter=10, resth=1e-10, max_kl=0.01,
           max_bt=10, accept=0.1, verbose=False):
    """One TRPO_Update (src/TRPO_Update.c:10-1011).  Returns a dict."""
    obs = _f64(obs)
    P = num_params(layers)
    th, b, x = np.zeros(P), np.zeros(P), np.zeros(P)
    scal = np.zeros(6)
    are = np.zeros(3 * max(max_bt, 1))
    ev = C.c_int(0)
    t = lib().oracle_update(len(layers), _ls(layers), acfunc.encode(), _f64(theta), obs, _f64(mean), _f64(action),
                            _f64(adv), _f64(std), obs.shape[0], damping, maxiter, resth, max_kl, max_bt, accept,
                            th, b, x, scal, are, C.byref(ev), 1 if verbose else 0)
    if t < 0:
        raise RuntimeError("oracle_update failed")
    k = ev.value
    return dict(theta=th, b=b, x=x, shs=scal[0], lagrange=scal[1], gnorm=scal[2], fval=scal[3], rate=scal[4],
                accepted=int(scal[5]), evaluated=k, actual=are[0:3 * k:3], expected=are[1:3 * k:3],
                ratio=are[2:3 * k:3], seconds=t)


def load_rollout(path, layers, n):
    """Every column of a data file: (obs, std_of_last_line, mean, action, adv)."""
    A = layers[-1]
    obs, std = np.zeros((n, layers[0])), np.zeros(A)
    mean, action, adv = np.zeros((n, A)), np.zeros((n, A)), np.zeros(n)
    if lib().oracle_load_rollout(path.encode(), len(layers), _ls(layers), n, obs, std, mean, action, adv):
        raise IOError(path)
    return obs, std, mean, action, adv


def baseline_evaluate(layers, acfunc, x, observ, target, num_ep, ep_len):
    """src/TRPO_Baseline.c:29-240.  x: PaddedParams (or NumParams) values.  Returns (f, g, predict)."""
    x = _f64(x)
    g = np.zeros(x.size)
    pred = np.zeros(num_ep * ep_len)
    f = lib().oracle_baseline_evaluate(len(layers), _ls(layers), acfunc.encode(), x, x.size, _f64(observ),
                                       _f64(target), num_ep, ep_len, g, pred)
    return f, g, pred
