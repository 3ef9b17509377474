#!/usr/bin/env python3
"""Phase split of k_chain_walk (timing build: -DFS2_PHASE_TIMING).

  python fast-slam_amd/build.py --variant timing -DFS2_PHASE_TIMING
  FS2_LIB=fast-slam_amd/lib/libfs2_timing.so python3 scripts/chain_timing.py
Runs the config-3 workload for 20 scans and prints wave 0's s_memtime cycles
per walk in each phase, the units walked and those evaluated term by term.
"""
import ctypes as C
import os
import sys

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
    f = fast_slam_2.FastSLAM2(N, rng="device", landmark_capacity=L + 64, verbose=False)
    bench.populate(f, N, L, 0, 0)
    fn = nat.load().fs2_debug_chain_times
    fn.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    out = (C.c_uint64 * 8)()
    for s in range(3):
        f.step(*syn.odometry(s), syn.scan_measurements(L, s, 0))
    f.synchronize()
    fn(out, 1)
    fin0 = nat.load().fs2_debug_finalize_times
    fin0.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    fin0((C.c_uint64 * 8)(), 1)
    for s in range(3, 23):
        f.step(*syn.odometry(s), syn.scan_measurements(L, s, 0))
    f.synchronize()
    fn(out, 0)
    calls = max(out[4], 1)
    names = ["scan over units", "batch loads", "walk", "post-pass (prefix)"]
    print(f"walks {out[4]}, units walked per walk {out[5] / calls:.1f}, term-by-term {out[6] / calls:.2f}")
    for k, nme in enumerate(names):
        print(f"{nme:<20} {out[k] / calls:10.0f} cycles per walk (~{out[k] / calls / 2400.0:.2f} us at 2.4 GHz)")
    f.close()
    # k_finalize: thread 0's stamps (fs2_resample.hip FS2_FIN), same scans
    fin = nat.load().fs2_debug_finalize_times
    fin.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    fo = (C.c_uint64 * 8)()
    fin(fo, 0)
    n = max(fo[7], 1)
    for k, nme in enumerate(["loads issued + numpy trees", "partials folded", "block_sum", "argmax + max",
                             "thread 0: chunk sums in order", "pose loads + record", "decision + stats"]):
        print(f"k_finalize {nme:<32} {fo[k] / n:10.0f} cycles per call")


if __name__ == "__main__":
    main()
