#!/usr/bin/env python3
"""Dump the normalised weights of the config-3 bench workload after a few scans
(gpurun_out/weights_s*.npy), to study the exact-order chain's unit mix offline."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fast-slam_amd")]


def main():
    import torch  # noqa: F401
    import fast_slam_2
    import fs2_synthetic as syn
    import bench
    N, L = 1_000_000, 500
    f = fast_slam_2.FastSLAM2(N, rng="device", seed=0, landmark_capacity=L + 40, verbose=False)
    bench.populate(f, N, L, 0, 0)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    for s in range(12):
        _, st = f.step(*syn.odometry(s), syn.scan_measurements(L, s, 0))
        w = f.get_state(lm_cap=0)[3]
        if s in (4, 5, 9, 10, 11):
            np.save(os.path.join(REPO, "gpurun_out", f"weights_s{s}.npy"), w)
        print(s, st.resampled, st.total_weight, st.n_eff, flush=True)
    f.close()


if __name__ == "__main__":
    main()
