#!/usr/bin/env python3
"""The per-scan tail alone (normalise, N_eff, resample, estimate) on saved weights:
one scan without measurements or motion on a handle holding only these weights
(tests/test_gpu_exact.py run_tail), so a kernel trace shows the tail's kernels on
exactly that weight pattern.  python scripts/tail_probe.py weights.npz [repeats]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))


def main():
    import torch  # noqa: F401
    import fast_slam_2
    w = np.load(sys.argv[1])["w"]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    N = len(w)
    for r in range(reps):
        f = fast_slam_2.FastSLAM2(N, reduce="exact", verbose=False)
        f.set_state(np.arange(N, dtype=float), np.zeros(N), np.zeros(N), w)
        _, st = f.step(0.0, 0.0, np.zeros((0, 2)), None, np.zeros(N), 0.37 / N)
        print(r, "resampled", st.resampled, "n_eff", st.n_eff, flush=True)
        f.close()


if __name__ == "__main__":
    main()
