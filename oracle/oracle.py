"""ctypes front-end of the C oracle (oracle/fs2_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Used by tests/ as the parity checker and by bench.py as the CPU baseline
("port").  Never imported by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_lp = C.POINTER(C.c_int64)


class OrcCfg(C.Structure):
    _fields_ = [("tr_noise", C.c_double), ("rot_noise", C.c_double), ("R", C.c_double * 4),
                ("gate", C.c_double), ("init_cov", C.c_double * 4), ("floor", C.c_double)]


class OrcState(C.Structure):
    _fields_ = [("n", C.c_int64), ("cap", C.c_int32), ("x", _dp), ("y", _dp), ("yaw", _dp),
                ("w", _dp), ("cnt", _ip), ("lm", _dp)]


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "fs2_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.orc_pymod.restype = C.c_double
        L.orc_pymod.argtypes = [C.c_double, C.c_double]
        L.orc_inv2.argtypes = [_dp, _dp]
        L.orc_mahalanobis2.argtypes = [_dp, _dp, _dp, _dp]
        L.orc_associate.argtypes = [_dp, _dp, C.c_int, C.c_double]
        L.orc_np_sum.restype = C.c_double
        L.orc_np_sum.argtypes = [_dp, C.c_int64]
        L.orc_normalize.restype = C.c_double
        L.orc_normalize.argtypes = [_dp, C.c_int64, C.c_double]
        L.orc_neff.restype = C.c_double
        L.orc_neff.argtypes = [_dp, C.c_int64]
        L.orc_resample_src.argtypes = [_dp, C.c_int64, C.c_double, _lp]
        L.orc_argmax_first.restype = C.c_int64
        L.orc_argmax_first.argtypes = [_dp, C.c_int64]
        L.orc_iterate.argtypes = [C.POINTER(OrcState), C.POINTER(OrcCfg), C.c_double, C.c_double,
                                  _dp, _dp, C.c_int32, _dp, C.c_double, _dp, _ip, _ip, _dp]
        L.orc_best_fit.argtypes = [_dp, _dp, C.c_int32, _dp, _dp]
        L.orc_icp.restype = C.c_int32
        L.orc_icp.argtypes = [_dp, C.c_int32, _dp, C.c_int32, C.c_int32, C.c_double, _dp, _dp]
        L.orc_correlate_reflect.argtypes = [_dp, C.c_int64, C.c_int64, _dp, C.c_int32, _dp]
        L.orc_gauss_pdf2.restype = C.c_double
        L.orc_gauss_pdf2.argtypes = [_dp, _dp]
        _lib = L
    return _lib


def _p(a, t=_dp):
    return a.ctypes.data_as(t)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def threads():
    """OpenMP worker threads of the oracle's particle loops (OMP_NUM_THREADS)."""
    return int(lib().orc_threads())


def set_threads(n):
    lib().orc_set_threads(int(n))


def pymod(a, b):
    return lib().orc_pymod(a, b)


def inv2(A):
    A = _f64(A).reshape(4)
    out = np.empty(4)
    if lib().orc_inv2(_p(A), _p(out)):
        raise np.linalg.LinAlgError("Singular matrix")
    return out.reshape(2, 2)


def mahalanobis(a, b, cov):
    a, b, cov = _f64(a), _f64(b), _f64(cov).reshape(4)
    out = np.empty(1)
    if lib().orc_mahalanobis2(_p(a), _p(b), _p(cov), _p(out)):
        raise np.linalg.LinAlgError("Singular matrix")
    return float(out[0])


def associate(obs, lm, gate):
    obs, lm = _f64(obs), _f64(lm).reshape(-1, 6)
    return int(lib().orc_associate(_p(obs), _p(lm), len(lm), float(gate)))


def np_sum(a):
    a = _f64(a)
    return lib().orc_np_sum(_p(a), a.size)


def normalize(w, floor=1e-5):
    w = _f64(w).copy()
    lib().orc_normalize(_p(w), w.size, floor)
    return w


def n_eff(w):
    w = _f64(w)
    return lib().orc_neff(_p(w), w.size)


def resample_src(w, u0):
    w = _f64(w)
    src = np.empty(w.size, dtype=np.int64)
    lib().orc_resample_src(_p(w), w.size, float(u0), _p(src, _lp))
    return src


def argmax_first(w):
    w = _f64(w)
    return int(lib().orc_argmax_first(_p(w), w.size))


def gauss_pdf2(nu, S):
    nu, S = _f64(nu), _f64(S).reshape(4)
    return lib().orc_gauss_pdf2(_p(nu), _p(S))


def best_fit(src, tgt):
    src, tgt = _f64(src), _f64(tgt)
    R, t = np.empty(4), np.empty(2)
    lib().orc_best_fit(_p(src), _p(tgt), len(src), _p(R), _p(t))
    return R.reshape(2, 2), t


def icp(src, tgt, max_iterations=100, threshold=1e-5):
    src, tgt = _f64(src), _f64(tgt)
    R, t = np.empty(4), np.empty(2)
    it = lib().orc_icp(_p(src), len(src), _p(tgt), len(tgt), max_iterations, threshold,
                       _p(R), _p(t))
    return R.reshape(2, 2), t, int(it)


def gaussian_weights(sigma, truncate=4.0):
    """scipy.ndimage._gaussian_kernel1d(sigma, 0, radius)[::-1] (numpy arithmetic)."""
    sd = float(sigma)
    radius = int(truncate * sd + 0.5)
    sigma2 = sigma * sigma
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / sigma2 * x ** 2)
    phi = phi / phi.sum()
    return phi[::-1].copy(), radius


def line_filter(points, sigma=0.1):
    pts = _f64(points)
    wts, r = gaussian_weights(sigma)
    out = np.empty_like(pts)
    for col in range(2):
        src = np.ascontiguousarray(pts[:, col])
        dst = np.empty_like(src)
        lib().orc_correlate_reflect(_p(src), len(src), 1, _p(wts), r, _p(dst))
        out[:, col] = dst
    return out


class OracleFilter:
    """Particle filter state held in the oracle's [N][cap][6] host layout."""

    def __init__(self, N, cap, tr_noise=0.0055, rot_noise=0.001, meas_noise=None, gate=8.0,
                 init_cov=0.1, floor=1e-5):
        R = np.array([[1e-3, 0.0], [0.0, 1e-3]]) if meas_noise is None else np.asarray(meas_noise)
        self.cfg = OrcCfg(tr_noise, rot_noise, (C.c_double * 4)(*R.reshape(4)), float(gate),
                          (C.c_double * 4)(init_cov, 0.0, 0.0, init_cov), floor)
        self.N, self.cap = N, cap
        self.x = np.zeros(N)
        self.y = np.zeros(N)
        self.yaw = np.zeros(N)
        self.w = np.full(N, 1.0 / N)
        self.cnt = np.zeros(N, dtype=np.int32)
        self.lm = np.zeros((N, cap, 6))

    def set_state(self, x, y, yaw, w, cnt, lm):
        self.x[:] = x
        self.y[:] = y
        self.yaw[:] = yaw
        self.w[:] = w
        self.cnt[:] = cnt
        k = min(self.cap, lm.shape[1])
        self.lm[:] = 0.0
        self.lm[:, :k] = lm[:, :k]

    def _st(self):
        return OrcState(self.N, self.cap, _p(self.x), _p(self.y), _p(self.yaw), _p(self.w),
                        _p(self.cnt, _ip), _p(self.lm))

    def iterate(self, rotation, translation, meas, noise, u0=0.0, observed=None):
        meas = _f64(meas).reshape(-1, 2)
        M = len(meas)
        obs = None if observed is None else _f64(observed).reshape(-1, 2)
        noise = _f64(noise)
        st = self._st()
        pose = np.empty(3)
        assoc = np.empty((max(M, 1), self.N), dtype=np.int32)
        rs = C.c_int32(0)
        ne = C.c_double(0)
        rc = lib().orc_iterate(C.byref(st), C.byref(self.cfg), float(rotation), float(translation),
                               _p(meas), None if obs is None else _p(obs), M, _p(noise),
                               float(u0), _p(pose), _p(assoc, _ip), C.byref(rs), C.byref(ne))
        if rc == -2:
            raise np.linalg.LinAlgError("Singular matrix")
        if rc != 0:
            raise RuntimeError(f"oracle iterate failed: {rc}")
        return pose, assoc[:M], bool(rs.value), ne.value
