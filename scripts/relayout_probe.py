#!/usr/bin/env python3
"""Does a long run's k_candidates slow down because its pages scatter over the
pool?  Config-3 handle, scans 0..S1-1; time scans S1-10..S1-1; re-import every
map in place (fs2_get_state -> fs2_set_state through device buffers: fresh pages
in import order, spatial layout of the whole map); time the next 10 scans.
Prints k_candidates / k_update ms per launch (library events) for both windows."""
import ctypes as C
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
    from fast_slam_2 import _native as nat
    torch.cuda.set_device(0)
    N, L = 1_000_000, 500
    S1 = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    cap = L + S1 + 30
    f = fast_slam_2.FastSLAM2(N, rng="device", seed=0, reduce="auto", landmark_capacity=cap, verbose=False)
    bench.populate(f, N, L, 0, 0)
    meas = lambda s: np.ascontiguousarray(syn.scan_measurements(L, s, 0), dtype=np.float64)

    def window(s0, s1, tag):
        f.set_profiling(True, every=1)
        p0 = f.profile()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opened = 0
        for s in range(s0, s1):
            _, st = f.step(*syn.odometry(s), meas(s))
            opened += st.pages_opened
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / (s1 - s0) * 1e3
        p1 = f.profile()
        fl = p1["filter_launches"] - p0["filter_launches"]
        el = p1["exact_launches"] - p0["exact_launches"]
        print(f"{tag}: scans {s0}..{s1 - 1}: {dt:.3f} ms/scan, k_candidates "
              f"{(p1['filter_ms'] - p0['filter_ms']) / max(fl, 1):.3f} ms, k_update "
              f"{(p1['exact_ms'] - p0['exact_ms']) / max(el, 1):.3f} ms, pages opened/particle "
              f"{opened / (N * (s1 - s0)):.2f}", flush=True)
        f.set_profiling(False)

    for s in range(S1 - 10):
        f.step(*syn.odometry(s), meas(s))
    window(S1 - 10, S1, "before")
    # re-import every map through device buffers, 100k particles at a time
    lib = f._lib
    t0 = time.perf_counter()
    K = 100_000
    for o in range(0, N, K):
        k = min(K, N - o)
        lm = torch.empty((k, cap, 6), dtype=torch.float64, device="cuda")
        cnt = torch.empty(k, dtype=torch.int32, device="cuda")
        nat.check(lib.fs2_get_state(f._h, o, k, None, None, None, None, cnt.data_ptr(),
                                    lm.data_ptr(), cap, nat.FS2_DEVICE), f._h)
        torch.cuda.synchronize()
        nat.check(lib.fs2_set_state(f._h, o, k, None, None, None, None, cnt.data_ptr(),
                                    lm.data_ptr(), cap, nat.FS2_DEVICE), f._h)
        del lm, cnt
    torch.cuda.synchronize()
    print(f"re-import: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    window(S1, S1 + 10, "after re-import")
    window(S1 + 10, S1 + 20, "later")
    f.close()


if __name__ == "__main__":
    main()
