#!/usr/bin/env python3
"""Per-phase wave time of k_update (timing build: -DFS2_PHASE_TIMING).

  FS2_LIB=fast-slam_amd/lib/libfs2_timing.so python3 scripts/phase_timing.py
Runs the config-3 workload (bench.populate) for a few scans and prints the
share of summed per-wave s_memtime cycles spent in each phase of k_update.
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))

PHASES = ["move+scalars", "phase A (exact assoc + EKF)", "B1 (own pages, copies)",
          "B2 (replay + stores)", "tail (appends)", "weights+scalar stores"]


def main():
    import torch
    import bench
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    torch.cuda.set_device(0)
    N, L = int(os.environ.get("N", 1_000_000)), 500
    f = fast_slam_2.FastSLAM2(N, rng="device", reduce="parallel", landmark_capacity=L + 64, verbose=False)
    bench.populate(f, f.n_local, L, 0, 0)
    lib = nat.load()
    fn = lib.fs2_debug_phase_times
    fn.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    out = (C.c_uint64 * 8)()
    meas = [np.ascontiguousarray(syn.scan_measurements(L, s, 0)) for s in range(12)]
    for s in range(2):
        f.step(*syn.odometry(s), meas[s])
    f.synchronize()
    fn(out, 1)
    for s in range(2, 12):
        f.step(*syn.odometry(s), meas[s])
    f.synchronize()
    fn(out, 1)
    tot = sum(out[:6])
    for k, name in enumerate(PHASES):
        print(f"{name:<32} {out[k] / max(tot, 1) * 100:6.1f} %   ({out[k] / 1e9:.3f} G wave-cycles)")
    f.close()


if __name__ == "__main__":
    main()
