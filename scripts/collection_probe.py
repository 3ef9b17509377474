#!/usr/bin/env python3
"""When do pool collections run at config 3?  The bench's handle and stream for
`--scans` scans; prints every scan whose collection count rose, with its host
time and the pool size, and the mean scan time with and without them.

  python3 scripts/collection_probe.py [--scans 60]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (sets up the package path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=60)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import fast_slam_2
    import fs2_synthetic as syn
    cfg = bench.CONFIGS["3"]
    N, L = cfg["N"], cfg["L"]
    f = fast_slam_2.FastSLAM2(N, rng="device", seed=0, reduce="auto", landmark_capacity=L + a.scans + 8,
                              verbose=False)
    bench.populate(f, f.n_local, L, 0, 0)
    coll = None
    plain, with_coll = [], []
    for s in range(a.scans):
        ms = np.ascontiguousarray(syn.scan_measurements(L, s, 0), dtype=np.float64)
        t0 = time.perf_counter()
        _, st = f.step(*syn.odometry(s), ms)
        dt = (time.perf_counter() - t0) * 1e3
        if coll is not None and st.collections > coll:
            with_coll.append(dt)
            print(f"scan {s}: collection #{st.collections} {dt:.3f} ms, pool {st.pool_pages} pages, "
                  f"resampled {st.resampled}", flush=True)
        else:
            plain.append(dt)
        coll = st.collections
    print(f"scans {a.scans}: collections {len(with_coll)}, mean scan without {np.mean(plain[3:]):.3f} ms, "
          f"with {np.mean(with_coll) if with_coll else float('nan'):.3f} ms", flush=True)
    f.close()


if __name__ == "__main__":
    main()
