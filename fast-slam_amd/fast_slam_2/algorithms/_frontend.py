"""Batched landmark front-end on the GPU (libfs2 fs2_frontend, fs2_frontend.hip).

LandmarkUtils.get_measurements_to_landmarks (reference
fast_slam_2/utils/landmark_utils.py:21-89) and HoughTransformation
(algorithms/hough_transformation.py:14-145) are thin wrappers over `run`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _native as nat
from .. import config
from .line_filter import gaussian_taps

DEVICE = 0
_KEYS = ("lines", "intersections", "clusters", "corners", "measurements")


def run(scans, sigma: float | None = 0.1, want=("measurements",), legacy: bool | None = None,
        device: int | None = None):
    """Run the front-end over a list of scans (each [P_b][2] points (x, y)).

    sigma: LineFilter sigma (None: points are already filtered, the identity).
    Returns {key: list of per-scan arrays} for the keys in `want` plus "counts"
    ([B][4]: lines, intersections, clusters, corners).
    """
    scans = [nat.f64(s, (-1, 2)) for s in scans]
    B = len(scans)
    offs = np.zeros(B + 1, np.int64)
    np.cumsum([len(s) for s in scans], out=offs[1:])
    pts = np.ascontiguousarray(np.concatenate(scans) if B else np.zeros((0, 2)))
    taps, radius = (np.ones(1), 0) if sigma is None else gaussian_taps(sigma)
    legacy = config.FRONTEND_NUMPY1_PROMOTION if legacy is None else legacy
    dev = DEVICE if device is None else device
    lib = nat.load()
    cap = 16
    while True:
        out = nat.fs2_frontend_out()
        out.cap = cap
        bufs = {}
        for k in want:
            bufs[k] = np.zeros((B, cap, 2), np.float32 if k == "lines" else np.float64)
            setattr(out, k, bufs[k].ctypes.data)
        counts = np.zeros((B, 4), np.int32)
        out.counts = counts.ctypes.data
        rc = lib.fs2_frontend(dev, B, offs.ctypes.data, pts.ctypes.data, nat.FS2_HOST, nat.dptr(taps),
                              radius, int(bool(legacy)), C.byref(out))
        need = 0
        for k in want:
            col = {"lines": 0, "intersections": 1, "clusters": 2}.get(k, 3)
            need = max(need, int(counts[:, col].max()) if B else 0)
        if rc == nat.FS2_ERR_ARG and need > cap:
            cap = need
            continue
        nat.check(rc)
        res = {"counts": counts}
        for k in want:
            col = {"lines": 0, "intersections": 1, "clusters": 2}.get(k, 3)
            res[k] = [bufs[k][b, :counts[b, col]].copy() for b in range(B)]
        return res
