"""ICP probe: time per 720-point alignment and iterations (bench config 4 scans); with a
-DFS2_PHASE_TIMING build also the cycles per phase of an iteration."""
import sys, time, os
sys.path.insert(0, "/root/repo/fast-slam_amd"); sys.path.insert(0, "/root/repo")
import numpy as np, torch
import fast_slam_2, fs2_synthetic as syn
scans = [syn.room_scan((0.03 * s, 0.0, 0.0), 720, 0, s) for s in range(12)]
for s in range(3):
    R, t, it = fast_slam_2.ICP.get_transformation_ex(scans[s], scans[s+1])
t0 = time.perf_counter(); its = []
for s in range(10):
    R, t, it = fast_slam_2.ICP.get_transformation_ex(scans[s], scans[s+1]); its.append(it)
dt = (time.perf_counter() - t0) / 10
print("icp us per call", dt * 1e6, "iterations", its)
# timing build (-DFS2_PHASE_TIMING): cycles per phase over the 10 timed calls
import ctypes as C
from fast_slam_2 import _native as nat
lib = nat.load()
if hasattr(lib, "fs2_debug_icp_phase_times"):
    out = (C.c_uint64 * 4)()
    lib.fs2_debug_icp_phase_times(out, 1)
    for s in range(10):
        fast_slam_2.ICP.get_transformation_ex(scans[s], scans[s + 1])
    lib.fs2_debug_icp_phase_times(out, 0)
    tot = sum(its)
    names = ["nn search", "centroid sums", "covariance sums", "transform update"]
    for k in range(4):
        print(f"{names[k]:18s} {out[k] / tot:10.0f} cycles per iteration")
