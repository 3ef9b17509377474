"""Point with heading (reference: fast_slam_2/models/directed_point.py)."""
from .point import Point


class DirectedPoint(Point):
    __slots__ = ("yaw",)

    def __init__(self, x: float, y: float, yaw: float):
        super().__init__(x, y)
        self.yaw = yaw

    def to_dict(self):
        return {"x": self.x, "y": self.y, "yaw": self.yaw}
