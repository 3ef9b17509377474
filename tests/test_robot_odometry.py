"""Robot.icp_odometry (reference robot.py:108-118) on the reference's own ICP
results: bit-identical (host arithmetic, no GPU)."""
import os

import numpy as np

from conftest import GOLDEN


def test_icp_odometry_matches_reference():
    from fast_slam_2.models.robot import Robot
    d = np.load(os.path.join(GOLDEN, "unit_robot_icp.npz"))
    for k in range(len(d["v"])):
        rot, tr = Robot.icp_odometry(d["R"][k], d["t"][k], float(d["v"][k]))
        assert rot == d["rotation"][k] and tr == d["translation"][k], k
