#!/usr/bin/env python3
"""How SURVEY §8d's synthetic stream behaves over long runs (CPU, C oracle):
per scan, the filter's yaw, the fraction of hit measurements that associate and
the mean map size.  The measurements are made for a robot at the origin while
the odometry turns the particles, so appends rise after ~30 scans.

  python3 scripts/workload_drift.py [scans]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "fast-slam_amd"), REPO]
import fs2_synthetic as syn  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main(scans=63, N=200, L=500):
    wl = syn.Workload(N, L, 0)
    x, y, yaw = wl.poses()
    o = orc.OracleFilter(N, L + 2 * scans)
    o.set_state(x, y, yaw, np.full(N, 1 / N), np.full(N, L), wl.maps())
    rng = np.random.default_rng(0)
    for s in range(scans):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        pose, assoc, _, _ = o.iterate(rot, tr, ms, rng.normal(0, 0.001 if rot else 0.0055, N),
                                      rng.uniform(0, 1 / N))
        if s % 6 == 0 or s == scans - 1:
            print(f"scan {s:3d}  yaw {pose[2]:.3f}  hits associated {(assoc[:3] >= 0).mean():.2f}  "
                  f"landmarks {o.cnt.mean():.1f}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 63)
