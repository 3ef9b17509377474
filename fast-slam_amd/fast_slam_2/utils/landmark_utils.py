"""LandmarkUtils (reference: fast_slam_2/utils/landmark_utils.py): front-end
(get_measurements_to_landmarks, :21-89), association (:92-117) and known-landmark
clustering (:120-144), all on the GPU."""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _native as nat
from .. import config


class LandmarkUtils:
    known_landmarks: list = []
    device = 0

    @staticmethod
    def associate_landmarks(observed_landmark, particle_landmarks):
        """First landmark in list order within the Mahalanobis gate; (None, None) if none."""
        L = len(particle_landmarks)
        if L == 0:
            return None, None
        lm = np.empty((L, 6))
        for j, l in enumerate(particle_landmarks):
            lm[j, 0], lm[j, 1] = l.x, l.y
            lm[j, 2:] = np.asarray(l.cov, dtype=np.float64).reshape(4)
        obs = np.array([observed_landmark.x, observed_landmark.y], dtype=np.float64)
        idx = C.c_int32()
        nat.check(nat.load().fs2_associate(LandmarkUtils.device, nat.dptr(obs), nat.dptr(lm), L,
                                           float(config.MAXIMUM_LANDMARK_DISTANCE), C.byref(idx)))
        if idx.value < 0:
            return None, None
        return particle_landmarks[idx.value], int(idx.value)

    @staticmethod
    def get_measurements_to_landmarks(scanned_points):
        """Measurements (distance, angle) to the corners observed in a scan
        (landmark_utils.py:21-36): LineFilter, Hough intersections, DBSCAN(0.5, 1)
        centres and the 0.1 m corner test on the GPU (fs2_frontend)."""
        from ..models.measurement import Measurement
        m = LandmarkUtils.get_measurements_batch([scanned_points])[0]
        return [Measurement(float(d), float(a)) for d, a in m]

    @staticmethod
    def get_measurements_batch(scans, sigma: float = 0.1):
        """Batched form: one [M_b][2] (distance, angle) array per scan, all scans in
        one device pass."""
        from ..algorithms import _frontend
        return _frontend.run(scans, sigma=sigma, want=("measurements",))["measurements"]

    @staticmethod
    def get_observed_landmarks(scanned_points):
        """Corners as Landmark objects (landmark_utils.py:39-64); coordinates are numpy
        float32 scalars (float64 with config.FRONTEND_NUMPY1_PROMOTION) as in the reference."""
        from ..algorithms import _frontend
        from ..models.landmark import Landmark
        c = _frontend.run([scanned_points], want=("corners",))["corners"][0]
        t = np.float64 if config.FRONTEND_NUMPY1_PROMOTION else np.float32
        return [Landmark(t(x), t(y)) for x, y in c]

    @staticmethod
    def update_known_landmarks(particles):
        """Known landmarks = DBSCAN(eps 0.5, min_samples int(0.7 * average map size)) centres
        over every particle's landmarks (landmark_utils.py:120-144).  Given
        FastSLAM2.particles, the clustering runs on the device-resident maps."""
        from ..models.landmark import Landmark
        fs = getattr(particles, "_filter", None)
        if fs is not None:
            cen = fs.cluster_landmarks(eps=0.5, min_fraction=0.7)
            if cen is None:
                return
        else:
            pts = [(lm.x, lm.y) for p in particles for lm in p.landmarks]
            min_samples = int(len(pts) / len(particles) * 0.7)
            if min_samples < 1:
                return
            from .geometry_utils import GeometryUtils
            cen = GeometryUtils.cluster_points(pts, eps=0.5, min_samples=min_samples)
        LandmarkUtils.known_landmarks = [Landmark(float(c[0]), float(c[1])) for c in cen]
