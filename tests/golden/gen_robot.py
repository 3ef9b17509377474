#!/usr/bin/env python3
"""Golden vectors for Robot.get_transformation_icp (reference
fast_slam_2/models/robot.py:93-120), made by running the reference here.

The reference's Robot talks to the JdeRobot simulator through `HAL`; a stub HAL
module feeds it synthetic laser scans of the 20 x 15 m room and a
fixed pose (EvaluationUtils.set_actual_pos reads it).  Only the outputs are
written: the previous scan as Robot.scan_environment built it (robot.py:31-55),
the target scan, the linear velocity v, the reference's (rotation, translation)
and the ICP result it came from.

Run:  python tests/golden/gen_robot.py   (writes tests/golden/unit_robot_icp.npz)
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

spec = importlib.util.spec_from_file_location(
    "fs2_synthetic", os.path.join(REPO, "fast-slam_amd", "fs2_synthetic.py"))
syn = importlib.util.module_from_spec(spec)
sys.modules["fs2_synthetic"] = syn
spec.loader.exec_module(syn)


class _Laser:
    def __init__(self, values):
        self.values = list(values)
        self.minRange = 0.2
        self.maxRange = 10.0
        self.timeStamp = 0


class _Pose:
    x, y, yaw = -1.0, 1.0, 0.0


hal = types.ModuleType("HAL")
hal._laser = _Laser(np.full(180, 5.0))
hal.getLaserData = lambda: hal._laser
hal.getPose3d = lambda: _Pose()
hal.setV = lambda v: None
hal.setW = lambda w: None
sys.modules["HAL"] = hal
sys.modules.setdefault("cv2", types.ModuleType("cv2"))
sys.path.insert(0, REF)
from fast_slam_2.models.robot import Robot  # noqa: E402
from fast_slam_2.algorithms.icp import ICP  # noqa: E402
from fast_slam_2.utils.evaluation_utils import EvaluationUtils  # noqa: E402


def ranges(pose, seed, scan):
    pts = syn.room_scan(pose, 180, seed=seed, scan=scan)
    return np.hypot(pts[:, 0], pts[:, 1])


def main():
    EvaluationUtils.try_to_initialize()      # offsets from the stub pose (set_actual_pos needs them)
    motions = [((0.03, 0.0, 0.0), 0.3), ((0.0, 0.0, 0.05), 0.0), ((0.06, 0.02, -0.03), 0.3),
               ((0.0, 0.0, -0.08), 0.0), ((0.05, 0.0, 0.02), 0.0)]
    prevs, tgts, vs, rot, tr, Rs, ts = [], [], [], [], [], [], []
    for c, (mv, v) in enumerate(motions):
        hal._laser = _Laser(ranges((0.0, 0.0, 0.0), 60 + c, 0))
        robot = Robot()
        prev = robot._Robot__prev_points.copy()
        hal._laser = _Laser(ranges(mv, 60 + c, 1))
        target = Robot.scan_environment()
        R, t = ICP.get_transformation(prev.copy(), target.copy())
        r_, t_ = robot.get_transformation_icp(target, v)
        P = 180
        prevs.append(np.pad(prev, ((0, P - len(prev)), (0, 0)), constant_values=np.nan))
        tgts.append(np.pad(target, ((0, P - len(target)), (0, 0)), constant_values=np.nan))
        vs.append(v)
        rot.append(float(r_))
        tr.append(float(t_))
        Rs.append(R)
        ts.append(t)
    np.savez_compressed(os.path.join(HERE, "unit_robot_icp.npz"),
                        prev=np.stack(prevs), target=np.stack(tgts),
                        n_prev=np.array([int(np.isfinite(p[:, 0]).sum()) for p in prevs]),
                        n_target=np.array([int(np.isfinite(p[:, 0]).sum()) for p in tgts]),
                        v=np.array(vs), rotation=np.array(rot), translation=np.array(tr),
                        R=np.stack(Rs), t=np.stack(ts), versions=np.array(repr(dict(numpy=np.__version__))))


if __name__ == "__main__":
    main()
