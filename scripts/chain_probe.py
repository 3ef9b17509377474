#!/usr/bin/env python3
"""The config-3 handle for 63 scans (bench's inputs): host time of every step and,
for steps far slower than the median, the weights the scan started from (the
exact chain's input is these times each particle's likelihoods) -> npz."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fast-slam_amd")]


def main():
    import torch
    import bench
    import fast_slam_2
    import fs2_synthetic as syn
    torch.cuda.set_device(0)
    N, L, S = 1_000_000, 500, int(sys.argv[1]) if len(sys.argv) > 1 else 63
    out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/chain_probe.npz"
    f = fast_slam_2.FastSLAM2(N, rng="device", seed=0, reduce="auto", landmark_capacity=L + S + 8, verbose=False)
    bench.populate(f, N, L, 0, 0)
    ms, keep = [], {}
    for s in range(S):
        w0 = f.get_state(0, N)[3]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, st = f.step(*syn.odometry(s), np.ascontiguousarray(syn.scan_measurements(L, s, 0), dtype=np.float64))
        dt = (time.perf_counter() - t0) * 1e3
        ms.append(dt)
        w1 = f.get_state(0, N)[3]
        nz0 = int((w0 == 0).sum())
        print(f"scan {s} {dt:8.3f} ms resampled {st.resampled} neff {st.n_eff:.4g} total {st.total_weight:.4g} "
              f"flags {st.error_flags} w0[0] {w0[0]:.3g} zeros {nz0} min>0 {w0[w0 > 0].min() if (w0 > 0).any() else 0:.3g} "
              f"first_nz {int(np.argmax(w0 > 0))}", flush=True)
        if dt > 5.0 and len(keep) < 3:
            keep[f"w_before_{s}"] = w0
            keep[f"w_after_{s}"] = w1
    np.savez(out, ms=np.array(ms), **keep)
    f.close()


if __name__ == "__main__":
    main()
