"""Helpers shared by the GPU tests: build a FastSLAM2 handle from a golden fixture."""
import numpy as np

import fast_slam_2
from fast_slam_2 import config


def configure(tr=0.0055, rot=0.001, meas_noise=1e-3, gate=8):
    config.TRANSLATION_NOISE = float(tr)
    config.ROTATION_NOISE = float(rot)
    config.MEASUREMENT_NOISE = np.eye(2) * float(meas_noise)
    config.MAXIMUM_LANDMARK_DISTANCE = gate


def from_fixture(d, reduce="sequential", capacity=64):
    tr, rot, mn = d["noise_cfg"]
    configure(tr, rot, mn, float(d["gate"]))
    f = fast_slam_2.FastSLAM2(int(d["N"]), reduce=reduce, record_assoc=True,
                              landmark_capacity=capacity, verbose=False)
    f.set_state(d["x"][0], d["y"][0], d["yaw"][0], d["w"][0], d["cnt"][0], d["lm"][0])
    return f


def close(a, b, rtol=1e-9, atol=1e-12):
    return np.allclose(a, b, rtol=rtol, atol=atol)
