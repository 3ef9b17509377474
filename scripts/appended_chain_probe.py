#!/usr/bin/env python3
"""Why a resampling scan of the appended-maps workload (bench.py appended_maps)
takes milliseconds in k_chain_walk / k_ranges: run the workload scan by scan and,
after the first resampling scan slower than 2 ms, save the normalised weights the
resample read (fs2_debug_weights, the other buffer set) and the sources' output
counts (fs2_debug_out_src) to gpurun_out/appended_slow_scan.npz."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))


def main():
    import torch
    torch.cuda.set_device(0)
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    N, L = 1_000_000, 500
    lib = nat.load()
    g = fast_slam_2.FastSLAM2(N, rng="device", seed=0, landmark_capacity=L + 40, verbose=False)
    nb = syn.buildup_scans(L)
    stream = [("build", s) for s in range(nb)] + [("run", s) for s in range(23)]
    w = np.empty(N)
    src = np.empty(N, dtype=np.int32)
    for kind, s in stream:
        if kind == "build":
            rot, tr, ms = 0.0, 0.0, syn.buildup_measurements(L, s, 0)
        else:
            (rot, tr), ms = syn.odometry(s), syn.scan_measurements(L, s, 0)
        t0 = time.perf_counter()
        _, st = g.step(rot, tr, np.ascontiguousarray(ms))
        dt = (time.perf_counter() - t0) * 1e3
        print(f"{kind} {s}: {dt:.3f} ms resampled {int(st.resampled)} n_eff {st.n_eff:.1f}", flush=True)
        if st.resampled and dt > 2.0:
            nat.check(lib.fs2_debug_weights(g._h, 1, w.ctypes.data), g._h)
            lib.fs2_debug_out_src(g._h, src.ctypes.data, N)
            np.savez_compressed(os.path.join(REPO, "gpurun_out", "appended_slow_scan.npz"), w=w, out_src=src,
                                kind=kind, scan=s, ms=dt, n_eff=st.n_eff)
            print("saved", flush=True)
            break
    g.close()


if __name__ == "__main__":
    main()
