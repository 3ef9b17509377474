#!/usr/bin/env python3
"""Time the landmark front-end (LandmarkUtils.get_measurements_to_landmarks,
landmark_utils.py:21-89) on the GPU: one 180-beam scan (latency, the
reference's per-loop call at jde_robots_main.py:34) and a batch of B scans in
one fs2_frontend call (throughput), next to the C oracle on the host (the
reference itself cannot run here: cv2 is absent).  Scenes: the L-shaped room of
fs2_synthetic at random poses.  Prints one JSON line.

  python3 scripts/bench_frontend.py [--batch 2000] [--beams 180]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fast-slam_amd")]


def scenes(n, P, seed=0):
    import fs2_synthetic as syn
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        pose = (rng.uniform(-5, 1.5), rng.uniform(-3.5, 4.5), rng.uniform(-np.pi, np.pi))
        pts = syn.polygon_scan(syn.L_ROOM, pose, P, rng)
        if len(pts) >= 10:
            out.append(pts)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2000)
    ap.add_argument("--beams", type=int, default=180)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-scans", type=int, default=100)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime in the process)
    from fast_slam_2 import LandmarkUtils
    from fast_slam_2.algorithms import _frontend
    from oracle import oracle as orc
    sc = scenes(args.batch, args.beams)
    one = sc[0]
    LandmarkUtils.get_measurements_to_landmarks(one)          # warm-up
    t = []
    for _ in range(20):
        t0 = time.perf_counter()
        LandmarkUtils.get_measurements_to_landmarks(one)
        t.append(time.perf_counter() - t0)
    single_ms = 1e3 * float(np.median(t))
    _frontend.run(sc, want=("measurements",))                 # warm-up (workspace growth)
    tb = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        r = _frontend.run(sc, want=("measurements",))
        tb.append(time.perf_counter() - t0)
    batch_s = float(min(tb))
    counts = r["counts"]
    # host C oracle on a sample (single thread)
    t0 = time.perf_counter()
    for s in sc[:args.cpu_scans]:
        orc.fe_extract(s)
    cpu_s = (time.perf_counter() - t0) / args.cpu_scans
    print(json.dumps({
        "workload": f"front-end, L-room, {args.beams}-beam scans",
        "single_scan_ms": single_ms,
        "batch": args.batch, "batch_ms": 1e3 * batch_s, "scans_per_s": args.batch / batch_s,
        "mean_counts": dict(zip(["lines", "intersections", "clusters", "corners"],
                                counts.mean(axis=0).round(2).tolist())),
        "cpu_oracle_ms_per_scan": 1e3 * cpu_s, "cpu_oracle_threads": 1}), flush=True)


if __name__ == "__main__":
    main()
