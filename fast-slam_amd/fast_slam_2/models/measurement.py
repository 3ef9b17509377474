"""Range/bearing observation of a landmark (reference: fast_slam_2/models/measurement.py)."""
import numpy as np


class Measurement:
    __slots__ = ("distance", "yaw")

    def __init__(self, distance: float, yaw: float):
        self.distance = distance
        self.yaw = yaw

    def as_vector(self):
        return np.array([self.distance, self.yaw])
