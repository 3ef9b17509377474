"""Particle: pose, weight and landmark map (reference: fast_slam_2/models/particle.py:11-20).

Host snapshot of one device particle; FastSLAM2.particles builds these lazily
and the FastSLAM2.particles setter uploads a list of them back to HBM.
"""
from .. import config
from .directed_point import DirectedPoint


class Particle(DirectedPoint):
    __slots__ = ("weight", "landmarks")

    def __init__(self, x: float, y: float, yaw: float):
        super().__init__(x, y, yaw)
        self.weight = 1.0 / config.NUM_PARTICLES
        self.landmarks = []

    def __str__(self):
        return (f"Particle: x: {self.x}, y: {self.y}, yaw: {self.yaw}, weight: {self.weight}, "
                f"landmarks: {self.landmarks}")
