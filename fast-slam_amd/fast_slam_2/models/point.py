"""2-D point (reference: fast_slam_2/models/point.py)."""
import numpy as np


class Point:
    __slots__ = ("x", "y")

    def __init__(self, x: float, y: float):
        self.x = x
        self.y = y

    def as_vector(self):
        return np.array([self.x, self.y])

    def to_dict(self):
        return {"x": self.x, "y": self.y}
