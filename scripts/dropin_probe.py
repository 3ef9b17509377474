"""Drop-in iterate() at BASELINE config 3 with numpy's stream drawn on the device:
per-scan wall time.  (profiles/r03_dropin_probe.txt also holds the host phases of
fs2_mt_draw from a build with FS2_MT_TIMING instrumentation, since removed.)"""
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))
import torch  # noqa: F401,E402
import bench  # noqa: E402
import fast_slam_2  # noqa: E402
import fs2_synthetic as syn  # noqa: E402
from fast_slam_2.models.measurement import Measurement  # noqa: E402

N, L, scans = 1000000, 500, 40
np.random.seed(0)
f = fast_slam_2.FastSLAM2(N, rng="numpy", seed=0, landmark_capacity=L + scans + 8, verbose=False)
bench.populate(f, N, L, 0, 0)
meas = [[Measurement(float(d), float(b)) for d, b in syn.scan_measurements(L, s, 0)] for s in range(scans)]
ts = []
for s in range(scans):
    t0 = time.perf_counter()
    f.iterate(*syn.odometry(s), meas[s])
    ts.append(time.perf_counter() - t0)
ts = np.array(ts[4:]) * 1e3
print(f"iterate ms/scan: median {np.median(ts):.3f} mean {ts.mean():.3f}", flush=True)
f.close()
