"""Python mirror of the reference's FVP/CG operator interface over libtrpo_mi355x.so.

Everything here is a ctypes view of the C ABI in include/trpo_mi355x.h -- the
same entry points the reference's C callers link against
(src/include/TRPO.h:81-101): ``NumParamsCalc``, ``FVP``, ``FVPFast``, ``CG``,
``FVP_FPGA``, ``CG_FPGA`` with a field-for-field ``TRPOparam`` -- plus the
in-memory :class:`Context`.  There is no CPU fallback: if the HIP library is
missing or no MI355X is visible, calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("TRPO_LIB") or os.path.join(PKG_DIR, "lib", "libtrpo_mi355x.so")
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "trpo_mi355x.h")

_lib = None
_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


class TRPOparam(C.Structure):
    """Layout of TRPOparam, src/include/TRPO.h:6-49 (passed BY VALUE)."""
    _fields_ = [
        ("ModelFile", C.c_char_p),
        ("BaselineFile", C.c_char_p),
        ("ResultFile", C.c_char_p),
        ("DataFile", C.c_char_p),
        ("NumLayers", C.c_size_t),
        ("AcFunc", C.c_char_p),
        ("LayerSize", C.POINTER(C.c_size_t)),
        ("NumSamples", C.c_size_t),
        ("CG_Damping", C.c_double),
        ("PaddedLayerSize", C.POINTER(C.c_size_t)),
        ("NumBlocks", C.POINTER(C.c_size_t)),
    ]


class TRPOError(RuntimeError):
    pass


def build(verbose: bool = False) -> str:
    """Compile lib/libtrpo_mi355x.so for gfx950 (hipcc cross-compiles; no GPU needed)."""
    import subprocess
    out = subprocess.run(["make", "-s", "-C", PKG_DIR, "-j4"], capture_output=not verbose, text=True)
    if out.returncode != 0:
        raise TRPOError("build failed:\n" + (out.stdout or "") + (out.stderr or ""))
    return LIB_PATH


def lib():
    """Load libtrpo_mi355x.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise TRPOError("libtrpo_mi355x.so not built: run trpo_amd.build() / make -C trpo-robot-control_amd")
    L = C.CDLL(LIB_PATH)
    sz = C.c_size_t
    P = C.POINTER
    L.NumParamsCalc.restype = sz
    L.NumParamsCalc.argtypes = [P(sz), sz]
    for name in ("FVPFast",):
        getattr(L, name).restype = C.c_double
        getattr(L, name).argtypes = [TRPOparam, _dp, _dp, sz]
    for name in ("FVP", "FVP_FPGA"):
        getattr(L, name).restype = C.c_double
        getattr(L, name).argtypes = [TRPOparam, _dp, _dp]
    for name in ("CG", "CG_FPGA"):
        getattr(L, name).restype = C.c_double
        getattr(L, name).argtypes = [TRPOparam, _dp, _dp, sz, C.c_double, sz]
    L.trpo_ctx_create.restype = C.c_void_p
    L.trpo_ctx_create.argtypes = [sz, P(sz), C.c_char_p, C.c_void_p, C.c_void_p, sz, C.c_void_p, C.c_double, C.c_int]
    L.trpo_ctx_destroy.restype = None
    L.trpo_ctx_destroy.argtypes = [C.c_void_p]
    for name in ("trpo_ctx_set_theta", "trpo_ctx_set_std", "trpo_ctx_upload_b", "trpo_ctx_upload_v",
                 "trpo_ctx_download_x", "trpo_ctx_download_z"):
        getattr(L, name).restype = C.c_int
        getattr(L, name).argtypes = [C.c_void_p, _dp]
    L.trpo_ctx_set_obs.restype = C.c_int
    L.trpo_ctx_set_obs.argtypes = [C.c_void_p, C.c_void_p, sz]
    L.trpo_ctx_set_damping.restype = C.c_int
    L.trpo_ctx_set_damping.argtypes = [C.c_void_p, C.c_double]
    L.trpo_ctx_num_params.restype = sz
    L.trpo_ctx_num_params.argtypes = [C.c_void_p]
    L.trpo_comm_unique_id.restype = C.c_int
    L.trpo_comm_unique_id.argtypes = [C.c_char_p]
    L.trpo_ctx_attach_comm.restype = C.c_int
    L.trpo_ctx_attach_comm.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p]
    L.trpo_ctx_attach_comm_timeout.restype = C.c_int
    L.trpo_ctx_attach_comm_timeout.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.c_long]
    L.trpo_ctx_comm_verify.restype = C.c_int
    L.trpo_ctx_comm_verify.argtypes = [C.c_void_p, C.c_long]
    L.trpo_ctx_wait.restype = C.c_int
    L.trpo_ctx_wait.argtypes = [C.c_void_p, C.c_long]
    L.trpo_ctx_comm_abort.restype = C.c_int
    L.trpo_ctx_comm_abort.argtypes = [C.c_void_p]
    L.trpo_group_create.restype = C.c_void_p
    L.trpo_group_create.argtypes = [C.c_int]
    L.trpo_group_destroy.restype = None
    L.trpo_group_destroy.argtypes = [C.c_void_p]
    L.trpo_ctx_attach_group.restype = C.c_int
    L.trpo_ctx_attach_group.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    L.trpo_ctx_comm_info.restype = C.c_int
    L.trpo_ctx_comm_info.argtypes = [C.c_void_p, P(C.c_int), P(C.c_int), P(C.c_int)]
    L.trpo_ctx_peer_handle.restype = C.c_int
    L.trpo_ctx_peer_handle.argtypes = [C.c_void_p, C.c_char_p]
    L.trpo_ctx_attach_peers.restype = C.c_int
    L.trpo_ctx_attach_peers.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p]
    L.trpo_ctx_attach_peers_local.restype = C.c_int
    L.trpo_ctx_attach_peers_local.argtypes = [C.c_void_p, C.c_int, C.c_int, P(C.c_void_p)]
    L.trpo_ctx_surrogate.restype = C.c_int
    L.trpo_ctx_surrogate.argtypes = [C.c_void_p, _dp, C.c_int, C.c_int, _dp]
    L.trpo_hip_runtime_path.restype = C.c_char_p
    L.trpo_hip_runtime_path.argtypes = []
    L.trpo_ctx_comm_backend.restype = C.c_char_p
    L.trpo_ctx_comm_backend.argtypes = [C.c_void_p]
    L.trpo_ctx_fvp.restype = C.c_double
    L.trpo_ctx_fvp.argtypes = [C.c_void_p, _dp, _dp]
    L.trpo_ctx_cg.restype = C.c_double
    L.trpo_ctx_cg.argtypes = [C.c_void_p, _dp, sz, C.c_double, _dp, C.c_int]
    L.trpo_ctx_cg_history.restype = C.c_int
    L.trpo_ctx_cg_history.argtypes = [C.c_void_p, _dp, _dp, sz, P(sz)]
    L.trpo_ctx_cg_status.restype = C.c_int
    L.trpo_ctx_cg_status.argtypes = [C.c_void_p, P(C.c_double), P(C.c_double), P(C.c_int)]
    for name in ("trpo_ctx_enqueue_fvp", "trpo_ctx_enqueue_fvp_kernel_only", "trpo_ctx_synchronize"):
        getattr(L, name).restype = C.c_int
        getattr(L, name).argtypes = [C.c_void_p]
    L.trpo_ctx_enqueue_cg.restype = C.c_int
    L.trpo_ctx_enqueue_cg.argtypes = [C.c_void_p, sz, C.c_double]
    L.trpo_ctx_time.restype = C.c_double
    L.trpo_ctx_time.argtypes = [C.c_void_p, C.c_int, C.c_int, sz, C.c_double]
    L.trpo_ctx_kernel_name.restype = C.c_char_p
    L.trpo_ctx_kernel_name.argtypes = [C.c_void_p]
    L.trpo_ctx_launch_geometry.restype = C.c_int
    L.trpo_ctx_launch_geometry.argtypes = [C.c_void_p, P(C.c_int), P(C.c_int), P(C.c_int)]
    L.TRPO_Update.restype = C.c_double
    L.TRPO_Update.argtypes = [TRPOparam, _dp, sz]
    L.trpo_ctx_set_rollout.restype = C.c_int
    L.trpo_ctx_set_rollout.argtypes = [C.c_void_p, _dp, _dp, _dp]
    L.trpo_ctx_update.restype = C.c_double
    L.trpo_ctx_update.argtypes = [C.c_void_p, sz, C.c_double, C.c_double, C.c_int, C.c_double, _dp, _dp, _dp,
                                  P(UpdateInfo), C.c_int]
    L.evaluate.restype = C.c_double
    L.evaluate.argtypes = [C.c_void_p, _dp, _dp, C.c_int, C.c_double]
    L.trpo_baseline_create.restype = C.c_void_p
    L.trpo_baseline_create.argtypes = [sz, P(sz), C.c_char_p, C.c_int]
    L.trpo_baseline_destroy.restype = None
    L.trpo_baseline_destroy.argtypes = [C.c_void_p]
    L.trpo_baseline_set_data.restype = C.c_int
    L.trpo_baseline_set_data.argtypes = [C.c_void_p, _dp, _dp, sz, sz]
    L.trpo_baseline_evaluate.restype = C.c_double
    L.trpo_baseline_evaluate.argtypes = [C.c_void_p, _dp, _dp, C.c_int, C.c_void_p]
    L.trpo_last_error.restype = C.c_char_p
    L.trpo_last_error.argtypes = []
    L.trpo_cache_clear.restype = None
    L.trpo_cache_clear.argtypes = []
    _lib = L
    rt = runtime_path()
    expect = built_runtime_dir()
    if rt and expect and not _same_dir(os.path.dirname(os.path.realpath(rt)), expect):
        # torch (or another HIP user) was imported first and its bundled runtime now serves this
        # library too.  Load this library before importing torch (tests/conftest.py and bench.py do).
        import warnings
        warnings.warn("libtrpo_mi355x.so runs on the HIP runtime %s, not the one it was built and linked "
                      "against (%s); import trpo_amd and call trpo_amd.lib() before importing torch" % (rt, expect),
                      RuntimeWarning, stacklevel=2)
    return L


def built_runtime_dir():
    """Directory of the libamdhip64 the library was linked and rpath'ed against (lib/build_info.json,
    written by the Makefile from its ROCM), resolved; None if unknown."""
    import json
    try:
        with open(os.path.join(os.path.dirname(LIB_PATH), "build_info.json")) as f:
            return os.path.realpath(json.load(f)["hip_runtime_dir"])
    except (OSError, ValueError, KeyError):
        return None


def _same_dir(a: str, b: str) -> bool:
    """Whole-path-component comparison of two resolved directories."""
    return os.path.normpath(os.path.realpath(a)).split(os.sep) == os.path.normpath(os.path.realpath(b)).split(os.sep)


def runtime_is_built_one() -> bool:
    """True when this process's HIP calls resolve to the runtime the library was built against."""
    expect = built_runtime_dir()
    return expect is None or _same_dir(os.path.dirname(os.path.realpath(runtime_path())), expect)


def runtime_path() -> str:
    """Path of the libamdhip64 this library's HIP calls resolve to (trpo_hip_runtime_path)."""
    return lib().trpo_hip_runtime_path().decode()


MAX_BACKTRACKS = 32
PEER_HANDLE_BYTES = 64      # include/trpo_mi355x.h TRPO_PEER_HANDLE_BYTES


class TRPOBaselineParam(C.Structure):
    """src/include/TRPO.h:50-77 (field-for-field)."""
    _fields_ = [("NumLayers", C.c_size_t), ("ObservSpaceDim", C.c_size_t), ("NumEpBatch", C.c_size_t),
                ("EpLen", C.c_size_t), ("NumSamples", C.c_size_t), ("NumParams", C.c_size_t),
                ("PaddedParams", C.c_int), ("AcFunc", C.c_char_p), ("LayerSizeBase", C.POINTER(C.c_size_t)),
                ("WBase", C.POINTER(C.POINTER(C.c_double))), ("BBase", C.POINTER(C.POINTER(C.c_double))),
                ("LayerBase", C.POINTER(C.POINTER(C.c_double))), ("GWBase", C.POINTER(C.POINTER(C.c_double))),
                ("GBBase", C.POINTER(C.POINTER(C.c_double))), ("GLayerBase", C.POINTER(C.POINTER(C.c_double))),
                ("Observ", C.POINTER(C.c_double)), ("Target", C.POINTER(C.c_double)),
                ("Predict", C.POINTER(C.c_double))]


def make_baseline_param(layers_base, acfunc: str, observ, target, num_ep: int, ep_len: int):
    """A TRPOBaselineParam as src/TRPO_MuJoCo.c:256-277 fills it (W/B arrays allocated, scratch NULL).
    The numpy arrays are kept alive on the returned object (._keep); .predict is the Predict array."""
    p = TRPOBaselineParam()
    observ = np.ascontiguousarray(observ, np.float64)
    target = np.ascontiguousarray(target, np.float64)
    n = num_ep * ep_len
    predict = np.zeros(n)
    npar = NumParamsCalc(list(layers_base)) - layers_base[-1]
    W = [np.zeros(layers_base[i] * layers_base[i + 1]) for i in range(len(layers_base) - 1)]
    B = [np.zeros(layers_base[i + 1]) for i in range(len(layers_base) - 1)]
    dpp = C.POINTER(C.c_double)
    warr = (dpp * len(W))(*[w.ctypes.data_as(dpp) for w in W])
    barr = (dpp * len(B))(*[b.ctypes.data_as(dpp) for b in B])
    ls = _sizes(layers_base)
    p.NumLayers, p.ObservSpaceDim, p.NumEpBatch, p.EpLen = len(layers_base), layers_base[0] - 1, num_ep, ep_len
    p.NumSamples, p.NumParams, p.PaddedParams = n, npar, (npar + 15) // 16 * 16
    p.AcFunc = acfunc.encode()
    p.LayerSizeBase = C.cast(ls, C.POINTER(C.c_size_t))
    p.WBase, p.BBase = C.cast(warr, C.POINTER(dpp)), C.cast(barr, C.POINTER(dpp))
    p.Observ, p.Target, p.Predict = observ.ctypes.data_as(dpp), target.ctypes.data_as(dpp), predict.ctypes.data_as(dpp)
    p._keep = (observ, target, predict, W, B, warr, barr, ls, p.AcFunc)
    p.predict, p.W, p.B = predict, W, B
    return p


def evaluate(param: TRPOBaselineParam, x, g) -> float:
    """src/TRPO_Baseline.c:29: the liblbfgs callback (g is written in place)."""
    return float(lib().evaluate(C.byref(param), np.ascontiguousarray(x, np.float64), g, len(g), 1.0))


class Baseline:
    """Device-resident value-baseline objective for L-BFGS (include/trpo_mi355x.h)."""

    def __init__(self, layers_base, acfunc: str, device: int = -1):
        self.layers = [int(v) for v in layers_base]
        self.np = NumParamsCalc(self.layers) - self.layers[-1]
        self._h = lib().trpo_baseline_create(len(self.layers), _sizes(self.layers), acfunc.encode(), device)
        if not self._h:
            raise TRPOError("trpo_baseline_create failed: " + last_error())
        self.n = 0

    def close(self):
        if getattr(self, "_h", None):
            lib().trpo_baseline_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_data(self, observ, target, num_ep: int, ep_len: int):
        rc = lib().trpo_baseline_set_data(self._h, np.ascontiguousarray(observ, np.float64),
                                          np.ascontiguousarray(target, np.float64), num_ep, ep_len)
        if rc < 0:
            raise TRPOError("set_data failed: " + last_error())
        self.n = num_ep * ep_len

    def evaluate(self, x, want_predict=False):
        """Returns (f, g) or (f, g, predict)."""
        x = np.ascontiguousarray(x, np.float64)
        g = np.zeros(x.size)
        pred = np.zeros(self.n) if want_predict else None
        f = lib().trpo_baseline_evaluate(self._h, x, g, x.size, pred.ctypes.data if want_predict else None)
        if f < 0:
            raise TRPOError("evaluate failed: " + last_error())
        return (f, g, pred) if want_predict else (f, g)


class UpdateInfo(C.Structure):
    """trpo_update_info (include/trpo_mi355x.h)."""
    _fields_ = [("shs", C.c_double), ("lagrange", C.c_double), ("gnorm", C.c_double), ("fval_before", C.c_double),
                ("expected_improve_rate", C.c_double), ("evaluated", C.c_int), ("accepted", C.c_int),
                ("actual", C.c_double * MAX_BACKTRACKS), ("expected", C.c_double * MAX_BACKTRACKS),
                ("ratio", C.c_double * MAX_BACKTRACKS), ("cg_iters", C.c_size_t)]


def last_error() -> str:
    return lib().trpo_last_error().decode(errors="replace")


# --------------------------------------------------------------------------
# reference-shaped entry points (src/include/TRPO.h:81-101)
# --------------------------------------------------------------------------
def _sizes(layers):
    arr = (C.c_size_t * len(layers))(*layers)
    return arr


def make_param(model_file: str, data_file: str, layers, acfunc: str, num_samples: int,
               cg_damping: float = 0.1) -> TRPOparam:
    """Build a TRPOparam as TRPOCpuCode.c does (src/TRPOCpuCode.c:88-95)."""
    p = TRPOparam()
    p._keep = (model_file.encode(), data_file.encode(), acfunc.encode(), _sizes(layers))
    p.ModelFile, p.DataFile, ac, ls = p._keep
    p.AcFunc = ac
    p.LayerSize = C.cast(ls, C.POINTER(C.c_size_t))
    p.NumLayers = len(layers)
    p.NumSamples = num_samples
    p.CG_Damping = cg_damping
    return p


def NumParamsCalc(layers) -> int:
    return int(lib().NumParamsCalc(_sizes(layers), len(layers)))


def FVPFast(param: TRPOparam, result: np.ndarray, inp: np.ndarray, num_threads: int = 1) -> float:
    return float(lib().FVPFast(param, result, inp, num_threads))


def FVP(param: TRPOparam, result: np.ndarray, inp: np.ndarray) -> float:
    return float(lib().FVP(param, result, inp))


def CG(param: TRPOparam, result: np.ndarray, b: np.ndarray, max_iter: int = 10, residual_th: float = 1e-10,
       num_threads: int = 1) -> float:
    return float(lib().CG(param, result, b, max_iter, residual_th, num_threads))


def TRPO_Update(param: TRPOparam, result: np.ndarray, num_threads: int = 1) -> float:
    """src/TRPO_Update.c:10-1011: result <- updated policy parameters."""
    return float(lib().TRPO_Update(param, result, num_threads))


def FVP_FPGA(param: TRPOparam, result: np.ndarray, inp: np.ndarray) -> float:
    return float(lib().FVP_FPGA(param, result, inp))


def CG_FPGA(param: TRPOparam, result: np.ndarray, b: np.ndarray, max_iter: int = 10,
            residual_th: float = 1e-10, num_threads: int = 1) -> float:
    return float(lib().CG_FPGA(param, result, b, max_iter, residual_th, num_threads))


# --------------------------------------------------------------------------
# in-memory context (include/trpo_mi355x.h part 2)
# --------------------------------------------------------------------------
class Context:
    """Device-resident FVP/CG problem: weights, observations and P-vectors stay in HBM."""

    def __init__(self, layers, acfunc: str, theta, obs, std, cg_damping: float = 0.1, device: int = -1,
                 precision: str = None):
        """precision: None (TRPO_PRECISION from the environment, default "fp32") or "fp32" / "fp64".
        "fp64" runs the FVP in fp64 on the fp64 MFMA -- the reference's own arithmetic."""
        L = lib()
        self.layers = [int(x) for x in layers]
        self.acfunc = acfunc
        self.P = NumParamsCalc(self.layers)
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        obs = np.ascontiguousarray(obs, dtype=np.float64)
        std = np.ascontiguousarray(std, dtype=np.float64)
        if theta.size != self.P or obs.ndim != 2 or obs.shape[1] != self.layers[0] or std.size != self.layers[-1]:
            raise ValueError("shape mismatch: theta %s obs %s std %s for layers %s"
                             % (theta.shape, obs.shape, std.shape, self.layers))
        self.n = obs.shape[0]
        saved = os.environ.get("TRPO_PRECISION")
        if precision is not None:                      # read by the library at context creation
            os.environ["TRPO_PRECISION"] = precision
        try:
            self._h = L.trpo_ctx_create(len(self.layers), _sizes(self.layers), acfunc.encode(),
                                        theta.ctypes.data, obs.ctypes.data, self.n, std.ctypes.data, cg_damping,
                                        device)
        finally:
            if precision is not None:
                if saved is None:
                    os.environ.pop("TRPO_PRECISION", None)
                else:
                    os.environ["TRPO_PRECISION"] = saved
        if not self._h:
            raise TRPOError("trpo_ctx_create failed: " + last_error())

    def close(self):
        if getattr(self, "_h", None):
            lib().trpo_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def _chk(rc, what):
        if rc < 0:
            raise TRPOError("%s failed (%s): %s" % (what, rc, last_error()))
        return rc

    def set_theta(self, theta):
        self._chk(lib().trpo_ctx_set_theta(self._h, np.ascontiguousarray(theta, np.float64)), "set_theta")

    def set_std(self, std):
        self._chk(lib().trpo_ctx_set_std(self._h, np.ascontiguousarray(std, np.float64)), "set_std")

    def set_obs(self, obs):
        obs = np.ascontiguousarray(obs, dtype=np.float64)
        self._chk(lib().trpo_ctx_set_obs(self._h, obs.ctypes.data, obs.shape[0]), "set_obs")
        self.n = obs.shape[0]

    def set_damping(self, d):
        self._chk(lib().trpo_ctx_set_damping(self._h, d), "set_damping")

    def attach_comm(self, rank: int, world: int, unique_id: bytes, timeout_ms: int = 0):
        """RCCL communicator; its init is bounded by timeout_ms (0: $TRPO_COMM_TIMEOUT_MS or 120 s)."""
        self._chk(lib().trpo_ctx_attach_comm_timeout(self._h, rank, world, unique_id, int(timeout_ms)), "attach_comm")

    def comm_verify(self, timeout_ms: int = 0):
        """Bounded self-check of the attached collective (all ranks together): raises TRPOError with
        .code -6 (no completion) / -7 (wrong sum) / -4 (collective error)."""
        rc = lib().trpo_ctx_comm_verify(self._h, int(timeout_ms))
        if rc < 0:
            err = TRPOError("comm_verify failed (%d): %s" % (rc, last_error()))
            err.code = rc
            raise err

    def wait(self, timeout_ms: int = 0):
        """Wait for the enqueued work at most timeout_ms (TRPOError with .code -6 on time-out)."""
        rc = lib().trpo_ctx_wait(self._h, int(timeout_ms))
        if rc < 0:
            err = TRPOError("wait failed (%d): %s" % (rc, last_error()))
            err.code = rc
            raise err

    def comm_abort(self):
        """Abandon the collective (RCCL abort / peer error flag); the context is then only good for close()."""
        return lib().trpo_ctx_comm_abort(self._h)

    def attach_group(self, group: "Group", rank: int):
        """Join an in-process host group as `rank` (call concurrently from one thread per rank)."""
        self._chk(lib().trpo_ctx_attach_group(self._h, group._h, rank), "attach_group")

    def peer_handle(self) -> bytes:
        """Open this rank's peer exchange window; returns its exported handle (PEER_HANDLE_BYTES)."""
        buf = C.create_string_buffer(PEER_HANDLE_BYTES)
        self._chk(lib().trpo_ctx_peer_handle(self._h, buf), "peer_handle")
        return buf.raw

    def attach_peers(self, rank: int, world: int, handles):
        """Attach the peer-window exchange (every rank concurrently): handles = the world's
        peer_handle() bytes in rank order."""
        blob = b"".join(bytes(h) for h in handles)
        if len(blob) != world * PEER_HANDLE_BYTES:
            raise ValueError("need %d handles of %d bytes" % (world, PEER_HANDLE_BYTES))
        self._chk(lib().trpo_ctx_attach_peers(self._h, rank, world, blob), "attach_peers")

    def attach_peers_local(self, rank: int, ctxs):
        """In-process peer exchange: ctxs = the contexts of all ranks in rank order, each with an open
        window (peer_handle()); call concurrently, one thread per rank."""
        arr = (C.c_void_p * len(ctxs))(*[c._h for c in ctxs])
        self._chk(lib().trpo_ctx_attach_peers_local(self._h, rank, len(ctxs), arr), "attach_peers_local")

    def surrogate(self, fullstep, k0=0, nk=1):
        """Line-search surrogate sums at theta + 0.5^(k0+j) fullstep, j < nk (all ranks)."""
        out = np.zeros(nk)
        self._chk(lib().trpo_ctx_surrogate(self._h, np.ascontiguousarray(fullstep, np.float64), k0, nk, out),
                  "surrogate")
        return out

    @property
    def comm_backend(self) -> str:
        return lib().trpo_ctx_comm_backend(self._h).decode()

    def comm_info(self):
        """dict(rank, world, replicas, backend): the communicator as the collective library reports it."""
        r, w, rep = C.c_int(0), C.c_int(0), C.c_int(0)
        self._chk(lib().trpo_ctx_comm_info(self._h, C.byref(r), C.byref(w), C.byref(rep)), "comm_info")
        return dict(rank=r.value, world=w.value, replicas=rep.value, backend=self.comm_backend)

    def fvp(self, v):
        out = np.zeros(self.P)
        self._chk(lib().trpo_ctx_fvp(self._h, np.ascontiguousarray(v, np.float64), out), "fvp")
        return out

    def cg(self, b, max_iter=10, residual_th=1e-10, verbose=False):
        x = np.zeros(self.P)
        self._chk(lib().trpo_ctx_cg(self._h, np.ascontiguousarray(b, np.float64), max_iter, residual_th, x,
                                    1 if verbose else 0), "cg")
        return x

    def cg_history(self, cap=1024):
        rr, xn, it = np.zeros(cap), np.zeros(cap), C.c_size_t(0)
        self._chk(lib().trpo_ctx_cg_history(self._h, rr, xn, cap, C.byref(it)), "cg_history")
        n = it.value + 1
        return rr[:n], xn[:n], it.value

    def cg_status(self):
        """The fp32 stall guard of the last cg() / update(): dict(ritz_residual = the smallest relative
        Ritz residual of the solve, orth_loss = the largest fraction of a new residual the
        reorthogonalisation removed, fp64_rerun = the solve was repeated in fp64)."""
        rz, o, r = C.c_double(0.0), C.c_double(0.0), C.c_int(0)
        self._chk(lib().trpo_ctx_cg_status(self._h, C.byref(rz), C.byref(o), C.byref(r)), "cg_status")
        return dict(ritz_residual=rz.value, orth_loss=o.value, fp64_rerun=bool(r.value))

    def set_rollout(self, mean, action, adv):
        """Mean [n][A], Action [n][A], Advantage [n] of this context's samples (TRPO_Update)."""
        A = self.layers[-1]
        mean = np.ascontiguousarray(mean, np.float64)
        action = np.ascontiguousarray(action, np.float64)
        adv = np.ascontiguousarray(adv, np.float64)
        if mean.size != self.n * A or action.size != self.n * A or adv.size != self.n:
            raise ValueError("rollout shape mismatch for n=%d A=%d" % (self.n, A))
        self._chk(lib().trpo_ctx_set_rollout(self._h, mean, action, adv), "set_rollout")

    def update(self, max_iter=10, residual_th=1e-10, max_kl=0.01, max_backtracks=10, accept_ratio=0.1,
               verbose=False):
        """One TRPO policy update (src/TRPO_Update.c:254-1007).  Returns a dict with the new
        parameters, the policy gradient b, the CG step x and the step-size / line-search values."""
        th, b, x = np.zeros(self.P), np.zeros(self.P), np.zeros(self.P)
        info = UpdateInfo()
        t = self._chk(lib().trpo_ctx_update(self._h, max_iter, residual_th, max_kl, max_backtracks, accept_ratio,
                                            th, b, x, C.byref(info), 1 if verbose else 0), "update")
        k = info.evaluated
        st = self.cg_status()
        return dict(theta=th, b=b, x=x, shs=info.shs, ritz_residual=st["ritz_residual"], orth_loss=st["orth_loss"],
                    fp64_rerun=st["fp64_rerun"], lagrange=info.lagrange, gnorm=info.gnorm,
                    fval=info.fval_before, rate=info.expected_improve_rate, accepted=info.accepted, evaluated=k,
                    actual=np.array(info.actual[:k]), expected=np.array(info.expected[:k]),
                    ratio=np.array(info.ratio[:k]), cg_iters=info.cg_iters, seconds=t)

    # device-resident hooks used by bench.py
    def upload_b(self, b):
        self._chk(lib().trpo_ctx_upload_b(self._h, np.ascontiguousarray(b, np.float64)), "upload_b")

    def upload_v(self, v):
        self._chk(lib().trpo_ctx_upload_v(self._h, np.ascontiguousarray(v, np.float64)), "upload_v")

    def enqueue_cg(self, max_iter=10, residual_th=0.0):
        self._chk(lib().trpo_ctx_enqueue_cg(self._h, max_iter, residual_th), "enqueue_cg")

    def enqueue_fvp(self):
        self._chk(lib().trpo_ctx_enqueue_fvp(self._h), "enqueue_fvp")

    def enqueue_fvp_kernel(self):
        self._chk(lib().trpo_ctx_enqueue_fvp_kernel_only(self._h), "enqueue_fvp_kernel")

    def synchronize(self):
        self._chk(lib().trpo_ctx_synchronize(self._h), "synchronize")

    def time_ms(self, what: int, reps: int, max_iter: int = 10, residual_th: float = 0.0) -> float:
        return self._chk(lib().trpo_ctx_time(self._h, what, reps, max_iter, residual_th), "time")

    def download_x(self):
        x = np.zeros(self.P)
        self._chk(lib().trpo_ctx_download_x(self._h, x), "download_x")
        return x

    def download_z(self):
        z = np.zeros(self.P)
        self._chk(lib().trpo_ctx_download_z(self._h, z), "download_z")
        return z

    @property
    def kernel_name(self) -> str:
        return lib().trpo_ctx_kernel_name(self._h).decode()

    @property
    def geometry(self):
        b, t, l = C.c_int(0), C.c_int(0), C.c_int(0)
        lib().trpo_ctx_launch_geometry(self._h, C.byref(b), C.byref(t), C.byref(l))
        return dict(blocks=b.value, threads=t.value, lds_bytes=l.value)


class Group:
    """In-process host-staged sharding group (include/trpo_mi355x.h trpo_group_*)."""

    def __init__(self, world: int):
        self._h = lib().trpo_group_create(world)
        if not self._h:
            raise TRPOError("trpo_group_create(%d) failed" % world)
        self.world = world

    def close(self):
        if getattr(self, "_h", None):
            lib().trpo_group_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    rc = lib().trpo_comm_unique_id(buf)
    if rc < 0:
        raise TRPOError("ncclGetUniqueId failed")
    return buf.raw


def cache_clear():
    lib().trpo_cache_clear()


def header_symbols(path: str = HEADER):
    """Function names declared in include/trpo_mi355x.h (for the export test)."""
    import re
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", txt)) - {"if", "defined", "sizeof"})
