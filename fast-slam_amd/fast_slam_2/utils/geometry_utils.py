"""Geometry helpers (reference: fast_slam_2/utils/geometry_utils.py)."""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from .. import _native as nat


class GeometryUtils:
    device = 0

    @staticmethod
    def mahalanobis_distance(position_a, position_b, covariance_matrix) -> float:
        """sqrt((b-a)^T inv(cov) (b-a)), bit-identical to the reference (geometry_utils.py:13-23)."""
        return float(GeometryUtils.mahalanobis_distances(
            np.reshape(position_a, (1, 2)), np.reshape(position_b, (1, 2)),
            np.reshape(covariance_matrix, (1, 2, 2)))[0])

    @staticmethod
    def mahalanobis_distances(a, b, cov) -> np.ndarray:
        """Batched form: a, b [K][2]; cov [K][2][2] -> [K]."""
        a, b, cov = nat.f64(a, (-1, 2)), nat.f64(b, (-1, 2)), nat.f64(cov, (-1, 4))
        out = np.empty(len(a))
        nat.check(nat.load().fs2_mahalanobis(GeometryUtils.device, nat.dptr(a), nat.dptr(b),
                                             nat.dptr(cov), len(a), nat.dptr(out)))
        return out

    @staticmethod
    def calculate_distance_and_angle(x: float, y: float) -> tuple[float, float]:
        """Measurement construction (geometry_utils.py:65-74); host-side by design."""
        return math.sqrt(x ** 2 + y ** 2), math.atan2(y, x)

    @staticmethod
    def cluster_points(point_lists, eps: float, min_samples: int):
        """DBSCAN(eps, min_samples) + cluster centres (geometry_utils.py:26-62) on the GPU:
        exact sklearn labels, centres as numpy means, in label order."""
        pts = nat.f64(np.asarray(point_lists, dtype=np.float64).reshape(-1, 2))
        centres, _ = GeometryUtils.dbscan(pts, eps, min_samples, labels=False)
        return [c for c in centres]

    @staticmethod
    def dbscan(points, eps: float, min_samples: int, labels: bool = True):
        """(centres [K][2], labels [n] or None) of sklearn DBSCAN(eps, min_samples)."""
        pts = nat.f64(np.asarray(points, dtype=np.float64).reshape(-1, 2))
        if len(pts) == 0:
            raise ValueError("Found array with 0 sample(s) (shape=(0, 2)) while a minimum of 1 is required")
        lib = nat.load()
        lab = np.empty(len(pts), dtype=np.int32) if labels else None
        cap = 64
        while True:
            cen = np.empty((cap, 2))
            k = C.c_int64()
            rc = lib.fs2_cluster_points(GeometryUtils.device, nat.ptr(pts), len(pts), float(eps),
                                        int(min_samples), nat.ptr(cen), cap, C.byref(k), nat.ptr(lab),
                                        nat.FS2_HOST)
            if rc == nat.FS2_ERR_ARG and k.value > cap:
                cap = int(k.value)
                continue
            nat.check(rc)
            return cen[:k.value].copy(), lab
