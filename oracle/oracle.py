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
# ORACLE_LIB selects another build of the same sources (the sanitizer build)
LIB_PATH = os.environ.get("ORACLE_LIB", os.path.join(HERE, "_build", "liboracle.so"))

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
    srcs = [os.path.join(HERE, f) for f in ("fs2_oracle.c", "fs2_frontend_oracle.c", "Makefile")]
    if force or not os.path.exists(LIB_PATH) or any(os.path.getmtime(LIB_PATH) < os.path.getmtime(s)
                                                    for s in srcs):
        target = os.path.relpath(LIB_PATH, HERE) if os.path.dirname(LIB_PATH).startswith(HERE) else ""
        subprocess.run(["make", "-s", "-C", HERE] + ([target] if target else []), check=True)
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
        _fp = C.POINTER(C.c_float)
        L.orc_np_sinf.restype = C.c_float
        L.orc_np_sinf.argtypes = [C.c_float]
        L.orc_np_cosf.restype = C.c_float
        L.orc_np_cosf.argtypes = [C.c_float]
        L.orc_fe_geom.argtypes = [_dp, C.c_int, _lp]
        L.orc_fe_raster.argtypes = [_dp, C.c_int, _lp, C.POINTER(C.c_uint8)]
        L.orc_fe_trig.argtypes = [C.c_int, C.c_float, _fp, _fp]
        L.orc_fe_hough.restype = C.c_int
        L.orc_fe_hough.argtypes = [C.POINTER(C.c_uint8), C.c_int, C.c_int, C.c_int, _fp, C.c_int]
        L.orc_fe_intersections.restype = C.c_int
        L.orc_fe_intersections.argtypes = [_fp, C.c_int, C.c_int64, C.c_int64, _fp, C.c_int]
        L.orc_fe_back.argtypes = [_fp, C.c_int, C.c_int64, C.c_int64, C.c_int, _dp]
        L.orc_fe_cluster1.restype = C.c_int
        L.orc_fe_cluster1.argtypes = [_dp, C.c_int, C.c_double, C.c_int, _dp]
        L.orc_fe_corners.restype = C.c_int
        L.orc_fe_corners.argtypes = [_dp, C.c_int, _dp, C.c_int, C.c_double, _dp]
        L.orc_fe_measure.argtypes = [_dp, C.c_int, C.c_int, _dp]
        L.orc_fe_extract.restype = C.c_int
        L.orc_fe_extract.argtypes = [_dp, C.c_int, _dp, C.c_int32, C.c_int, _dp, C.c_int, _ip]
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


# ------------------------------------------------------------- front-end ---
# LandmarkUtils.get_measurements_to_landmarks (landmark_utils.py:21-89) and
# HoughTransformation (hough_transformation.py:14-145), fs2_frontend_oracle.c.

def _f32p(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def np_sinf(x):
    return np.float32(lib().orc_np_sinf(float(np.float32(x))))


def np_cosf(x):
    return np.float32(lib().orc_np_cosf(float(np.float32(x))))


def fe_geom(points):
    pts = _f64(points)
    g = np.zeros(4, np.int64)
    lib().orc_fe_geom(_p(pts), len(pts), _p(g, _lp))
    return [int(v) for v in g]


def fe_image(points):
    """The uint8 image HoughTransformation.__create_hough_transformation_image draws."""
    pts = _f64(points)
    g = np.array(fe_geom(pts), np.int64)
    img = np.zeros((int(g[3]), int(g[2])), np.uint8)
    lib().orc_fe_raster(_p(pts), len(pts), _p(g, _lp), img.ctypes.data_as(C.POINTER(C.c_uint8)))
    return img, [int(v) for v in g]


def fe_hough(img, threshold=80):
    """cv2.HoughLines(img, 1, np.pi / 180, threshold): float32 [K][2] (rho, theta)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    ip = img.ctypes.data_as(C.POINTER(C.c_uint8))
    K = lib().orc_fe_hough(ip, w, h, threshold, None, 0)
    lines = np.zeros((K, 2), np.float32)
    if K:
        lib().orc_fe_hough(ip, w, h, threshold, _f32p(lines), K)
    return lines


def fe_intersections(lines, width, height):
    lines = np.ascontiguousarray(lines, dtype=np.float32).reshape(-1, 2)
    K = len(lines)
    n = lib().orc_fe_intersections(_f32p(lines), K, width, height, None, 0)
    out = np.zeros((n, 2), np.float32)
    if n:
        lib().orc_fe_intersections(_f32p(lines), K, width, height, _f32p(out), n)
    return out


def fe_back(isect, off_x, off_y, legacy=False):
    isect = np.ascontiguousarray(isect, dtype=np.float32).reshape(-1, 2)
    out = np.zeros((len(isect), 2))
    lib().orc_fe_back(_f32p(isect), len(isect), off_x, off_y, int(legacy), _p(out))
    return out


def fe_cluster1(points, eps=0.5, legacy=False):
    pts = _f64(points).reshape(-1, 2)
    out = np.zeros((max(len(pts), 1), 2))
    K = lib().orc_fe_cluster1(_p(pts), len(pts), eps, int(legacy), _p(out))
    return out[:K]


def fe_corners(centres, scan, threshold=0.1):
    c = _f64(centres).reshape(-1, 2)
    sc = _f64(scan).reshape(-1, 2)
    out = np.zeros((max(len(c), 1), 2))
    m = lib().orc_fe_corners(_p(c), len(c), _p(sc), len(sc), threshold, _p(out))
    return out[:m]


def fe_measure(corners, legacy=False):
    c = _f64(corners).reshape(-1, 2)
    out = np.zeros((len(c), 2))
    lib().orc_fe_measure(_p(c), len(c), int(legacy), _p(out))
    return out


def fe_extract(points, sigma=0.1, legacy=False):
    """Measurements (distance, angle) [M][2] and counts (lines, intersections,
    clusters, corners) for one scan."""
    pts = _f64(points).reshape(-1, 2)
    wts, r = gaussian_weights(sigma)
    cap = 4096
    out = np.zeros((cap, 2))
    counts = np.zeros(4, np.int32)
    m = lib().orc_fe_extract(_p(pts), len(pts), _p(wts), r, int(legacy), _p(out), cap, _p(counts, _ip))
    if m < 0:
        raise MemoryError("front-end oracle allocation failed")
    return out[:min(m, cap)].copy(), counts


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
