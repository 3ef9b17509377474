"""Robot's ICP odometry (reference fast_slam_2/models/robot.py:93-120), without the
simulator.

The reference Robot reads the laser and drives the motors through the JdeRobot
simulator (HAL: scan_environment, move), which this build does not replace
(SURVEY.md §2).  What the hot path needs from it is the step that turns two
consecutive scans into the (rotation, translation) odometry fed to
FastSLAM2.iterate: ICP between the previous and the current scan (on the GPU,
algorithms/icp.py), then translation only while the robot drives (v != 0) and
rotation only while it turns (robot.py:108-118).
"""
from __future__ import annotations

import numpy as np

from ..algorithms.icp import ICP
from .directed_point import DirectedPoint


class Robot(DirectedPoint):
    __slots__ = ("_prev_points",)

    def __init__(self, x=0.0, y=0.0, yaw=0.0, prev_points=None):
        """prev_points: the scan the first ICP aligns from (the reference takes it from
        the laser in __init__, robot.py:25-28)."""
        super().__init__(x, y, yaw)
        self._prev_points = None if prev_points is None else np.asarray(prev_points, dtype=np.float64)

    @staticmethod
    def icp_odometry(rotation_matrix, translation_vector, v: float):
        """(rotation, translation) from an ICP result (robot.py:108-118): v != 0 keeps
        |t| and drops the rotation, v == 0 keeps -atan2(R10, R00) and drops t."""
        if v != 0:
            return 0, np.linalg.norm(translation_vector)
        return -np.arctan2(rotation_matrix[1, 0], rotation_matrix[0, 0]), 0

    def get_transformation_icp(self, target_points, v: float):
        """Robot.get_transformation_icp (robot.py:93-120): ICP from the previous scan to
        target_points, which become the previous scan; returns (rotation, translation)."""
        if self._prev_points is None:
            raise ValueError("Robot has no previous scan: pass prev_points")
        rotation_matrix, translation_vector = ICP.get_transformation(self._prev_points, target_points)
        self._prev_points = np.asarray(target_points, dtype=np.float64)
        return Robot.icp_odometry(rotation_matrix, translation_vector, v)

    def submit_icp(self, target_points):
        """The same alignment enqueued on the device's ICP stream (fs2_icp_submit), so
        that it runs beside the current filter update; finish with
        Robot.icp_odometry(*ticket.result()[:2], v)."""
        if self._prev_points is None:
            raise ValueError("Robot has no previous scan: pass prev_points")
        ticket = ICP.submit(self._prev_points, target_points)
        self._prev_points = np.asarray(target_points, dtype=np.float64)
        return ticket
