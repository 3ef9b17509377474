"""Drop-in iterate() at config 3 (N = 1e6, L = 500, numpy's stream drawn on the
device): the deferred draw (fs2_mt_draw_deferred, what the shim does) against the
synchronous one (fs2_mt_draw, then fs2_iterate), and device Philox (step) for
scale, each on a fresh handle from the same state; median ms per scan over scans
4..N.  Prints one JSON line.  Run on the GPU box."""
import ctypes as C
import json
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
from fast_slam_2 import _native as nat  # noqa: E402
from fast_slam_2 import config  # noqa: E402
from fast_slam_2.models.measurement import Measurement  # noqa: E402

N, L, scans = 1000000, 500, 24


def run(mode):
    np.random.seed(0)
    f = fast_slam_2.FastSLAM2(N, rng="numpy" if mode != "philox" else "device", seed=0,
                              landmark_capacity=L + scans + 8, verbose=False)
    bench.populate(f, N, L, 0, 0)
    lib = f._lib
    meas = [[Measurement(float(d), float(b)) for d, b in syn.scan_measurements(L, s, 0)] for s in range(scans)]
    arr = [np.ascontiguousarray(syn.scan_measurements(L, s, 0), dtype=np.float64) for s in range(scans)]
    mi, ma, mu = nat.fs2_mt_state(), nat.fs2_mt_state(), nat.fs2_mt_state()
    pose = np.empty(3)
    st = nat.fs2_iter_stats()
    ts = []
    for s in range(scans):
        rot, tr = syn.odometry(s)
        t0 = time.perf_counter()
        if mode == "deferred":
            f.iterate(rot, tr, meas[s])
        elif mode == "philox":
            f.step(rot, tr, arr[s])
        else:
            mi_ = nat.fs2_mt_state.from_numpy(np.random.get_state())
            sigma = config.ROTATION_NOISE if rot != 0 else config.TRANSLATION_NOISE
            nat.check(lib.fs2_mt_draw(f._h, C.byref(mi_), float(sigma), C.byref(ma), C.byref(mu), None), f._h)
            nat.check(lib.fs2_iterate(f._h, float(rot), float(tr), nat.ptr(arr[s]), None, arr[s].shape[0], None,
                                      None, nat.dptr(pose), C.byref(st)), f._h)
            np.random.set_state((mu if st.resampled else ma).to_numpy())
        ts.append(time.perf_counter() - t0)
    f.close()
    return float(np.median(np.array(ts[4:]) * 1e3))


out = [(m, run(m)) for m in ("philox", "deferred", "sync", "deferred")]
print(json.dumps(out), flush=True)
