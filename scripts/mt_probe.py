"""Time fs2_mt_draw (numpy's legacy stream drawn on the GPU) at N particles:
wall time per draw, and the drop-in iterate() split (draw vs scan) -- run under
rocprofv3 --kernel-trace --stats for the kernels' share."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fast-slam_amd"))
import torch  # noqa: F401,E402
import fast_slam_2  # noqa: E402
from fast_slam_2 import _native as nat  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
f = fast_slam_2.FastSLAM2(N, rng="numpy", verbose=False, landmark_capacity=8)
lib = nat.load()
np.random.seed(0)
mi, ma, mu, u0 = nat.fs2_mt_state(), nat.fs2_mt_state(), nat.fs2_mt_state(), C.c_double()
ts = []
for r in range(reps + 2):
    t0 = time.perf_counter()
    C.pointer(mi)[0] = nat.fs2_mt_state.from_numpy(np.random.get_state())
    nat.check(lib.fs2_mt_draw(f._h, C.byref(mi), 0.0055, C.byref(ma), C.byref(mu), C.byref(u0)), f._h)
    np.random.set_state(ma.to_numpy())
    ts.append(time.perf_counter() - t0)
ts = np.array(ts[2:]) * 1e3
print(f"N={N} fs2_mt_draw wall ms: median {np.median(ts):.3f} min {ts.min():.3f} max {ts.max():.3f}")
t0 = time.perf_counter()
for r in range(3):
    np.random.normal(0, 0.0055, size=N)
print(f"numpy normal(size=N) ms: {(time.perf_counter() - t0) / 3 * 1e3:.3f}")
f.close()
