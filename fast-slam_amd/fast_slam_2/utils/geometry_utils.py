"""Geometry helpers (reference: fast_slam_2/utils/geometry_utils.py)."""
from __future__ import annotations

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
        raise NotImplementedError(
            "GeometryUtils.cluster_points (DBSCAN, geometry_utils.py:26-62) is outside the "
            "particle-update hot path (SURVEY.md §8f, NEXT)")
