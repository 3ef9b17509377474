#!/usr/bin/env python3
"""Phase split of the per-scan tail kernels (timing build: -DFS2_PHASE_TIMING).

  python fast-slam_amd/build.py --variant timing -DFS2_PHASE_TIMING
  FS2_LIB=fast-slam_amd/lib/libfs2_timing.so python3 scripts/tail_timing.py
Runs the config-3 bench workload (3 warm-up + 20 scans) and prints, per scan,
workgroup 0 / thread 0's s_memrealtime intervals (100 MHz) inside k_chain_units,
k_normalize_chunks and k_finalize, and k_chain_walk's and k_finalize's own
s_memtime phase splits.
"""
import ctypes as C
import os
import sys

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
    lib = nat.load()
    tail = lib.fs2_debug_tail_times
    tail.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    out = (C.c_uint64 * 32)()
    for s in range(3):
        f.step(*syn.odometry(s), syn.scan_measurements(L, s, 0))
    f.synchronize()
    tail(out, 1)
    res = 0
    S = 20
    for s in range(3, 3 + S):
        _, st = f.step(*syn.odometry(s), syn.scan_measurements(L, s, 0))
        res += st.resampled
    f.synchronize()
    tail(out, 0)
    f.close()
    us = [v / 100.0 / S for v in out]          # 100 MHz ticks -> us, per scan
    print(f"{S} scans, {res} resampled; workgroup 0 / thread 0, us per scan (chain_units runs twice on a "
          f"resampling scan)")
    rows = [("k_chain_units: estimate loads + block sum", 0), ("k_chain_units: unit classification", 1),
            ("k_chain_units: group scan + stores", 2),
            ("k_normalize_chunks: workgroup 0 (to its partials)", 16),
            ("k_finalize_chunked: partial loads", 24), ("k_finalize_chunked: reductions + record + decision", 25),
            ("k_finalize_chunked: publication", 26)]
    for name, k in rows:
        print(f"{name:<52} {us[k]:8.2f}")


if __name__ == "__main__":
    main()
