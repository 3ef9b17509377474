#!/usr/bin/env python3
"""Time LandmarkUtils.update_known_landmarks (landmark_utils.py:120-144) on the
device-resident maps of a FastSLAM2 at BASELINE sizes (synthetic maps of
bench.populate: N particles x L landmarks, 6 m grid, 2 cm jitter), and the
reference CPU path (sklearn DBSCAN + numpy, here a 1000-particle sample).

  python3 scripts/bench_cluster.py [--particles 1000000] [--landmarks 500]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fast-slam_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=1_000_000)
    ap.add_argument("--landmarks", type=int, default=500)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-particles", type=int, default=1000)
    args = ap.parse_args()
    import torch
    import bench
    import fast_slam_2
    torch.cuda.set_device(0)
    N, L = args.particles, args.landmarks
    f = fast_slam_2.FastSLAM2(N, rng="device", landmark_capacity=L + 8, verbose=False)
    bench.populate(f, N, L, 0, 0)
    f.synchronize()
    cen = f.cluster_landmarks()                     # warm-up
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        cen = f.cluster_landmarks()
        times.append(time.perf_counter() - t0)
    out = {"workload": f"update_known_landmarks N={N} L={L}", "points": N * L,
           "clusters": int(len(cen)), "gpu_ms": 1e3 * min(times)}
    # reference CPU path on a sample (sklearn DBSCAN over n*L points + numpy means)
    try:
        from sklearn.cluster import DBSCAN
        n = min(args.cpu_particles, N)
        x, y, yaw, w, cnt, lm = f.get_state(0, n)
        pts = lm[:, :L, 0:2].reshape(-1, 2)
        t0 = time.perf_counter()
        db = DBSCAN(eps=0.5, min_samples=int(len(pts) / n * 0.7)).fit(pts)
        labs = db.labels_
        cpu_cen = [pts[labs == k].mean(axis=0) for k in set(labs) if k != -1]
        out["cpu_sample"] = {"particles": n, "points": int(len(pts)), "seconds": time.perf_counter() - t0,
                             "clusters": len(cpu_cen), "kind": "sklearn DBSCAN (reference path), 1 process"}
    except ImportError:
        out["cpu_sample"] = None
    print(json.dumps(out), flush=True)
    f.close()


if __name__ == "__main__":
    main()
