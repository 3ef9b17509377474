"""Landmark: mean and 2x2 covariance (reference: fast_slam_2/models/landmark.py:13-21).

On the device a particle's landmarks live in HBM pages; these
objects are host snapshots produced by FastSLAM2.particles.
"""
import numpy as np

from .point import Point

DEFAULT_COV = ((0.1, 0.0), (0.0, 0.1))


class Landmark(Point):
    __slots__ = ("cov",)

    def __init__(self, x: float, y: float, cov=None):
        super().__init__(x, y)
        self.cov = np.array(DEFAULT_COV) if cov is None else cov

    def __str__(self):
        return f"Landmark ID: x: {self.x}, y: {self.y}, Covariance: {self.cov}"
