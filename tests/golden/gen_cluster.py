#!/usr/bin/env python3
"""Golden fixtures for the known-landmark clustering.

Runs the reference's own GeometryUtils.cluster_points
(fast_slam_2/utils/geometry_utils.py:26-62, sklearn DBSCAN + numpy mean) and
LandmarkUtils.update_known_landmarks (fast_slam_2/utils/landmark_utils.py:120-144)
in this container (reference imported with empty HAL / cv2 stubs, as in
gen_golden.py) and records their outputs, plus sklearn's per-point labels.
Nothing from the reference is copied; only outputs on seeded inputs are saved.

Run:  python tests/golden/gen_cluster.py   (writes tests/golden/cluster_cases.npz)
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def import_reference():
    sys.modules.setdefault("HAL", types.ModuleType("HAL"))
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, REF)
    from fast_slam_2 import GeometryUtils, Landmark, LandmarkUtils, Particle
    return GeometryUtils, Landmark, LandmarkUtils, Particle


def cases(rng):
    out = []
    # blobs + uniform noise
    blobs = np.concatenate([rng.normal(c, 0.15, (400, 2)) for c in ([0, 0], [3, 1], [-2, 4])])
    out.append(("blobs_noise", np.concatenate([blobs, rng.uniform(-5, 7, (600, 2))]), 0.5, 10))
    # two blobs joined by a sparse bridge: border points in reach of both clusters
    a = rng.normal([0, 0], 0.1, (200, 2))
    b = rng.normal([1.6, 0], 0.1, (200, 2))
    bridge = np.stack([np.linspace(0.3, 1.3, 9), rng.normal(0, 0.02, 9)], 1)
    out.append(("bridge", np.concatenate([bridge, b, a]), 0.5, 12))
    # a lone border point between two separate clusters (lowest label wins)
    for ms in (30, 100):
        a2 = rng.normal([0, 0], 0.08, (300, 2))
        b2 = rng.normal([1.4, 0], 0.08, (300, 2))
        out.append((f"border_ms{ms}", np.concatenate([b2, [[0.7, 0.0]], a2]), 0.5, ms))
    # exact-eps spacing: lattice at 0.5 (distance == eps is a neighbour)
    g = np.stack(np.meshgrid(np.arange(8) * 0.5, np.arange(6) * 0.5), -1).reshape(-1, 2)
    out.append(("lattice_eps", np.concatenate([g, g[:5] + [10, 10]]), 0.5, 5))
    # duplicates and a single dense cluster
    d = np.repeat(rng.normal(0, 0.05, (30, 2)), 7, axis=0)
    out.append(("duplicates", d[rng.permutation(len(d))], 0.5, 20))
    # all noise (no cluster)
    out.append(("all_noise", rng.uniform(-50, 50, (300, 2)), 0.5, 4))
    # far-apart coordinates, small and large magnitudes
    far = np.concatenate([rng.normal([1e4, -3e3], 0.1, (150, 2)), rng.normal([-2e3, 5e4], 0.1, (150, 2)),
                          rng.normal([0, 0], 0.1, (150, 2))])
    out.append(("far", far, 0.5, 30))
    return out


def main():
    GeometryUtils, Landmark, LandmarkUtils, Particle = import_reference()
    from sklearn.cluster import DBSCAN
    import sklearn
    rng = np.random.default_rng(2024)
    data = {"versions": np.array([f"numpy={np.__version__}", f"sklearn={sklearn.__version__}"])}
    names = []
    for name, pts, eps, ms in cases(rng):
        centres = GeometryUtils.cluster_points([tuple(p) for p in pts], eps=eps, min_samples=ms)
        labels = DBSCAN(eps=eps, min_samples=ms).fit(pts).labels_
        data[f"{name}_points"] = pts
        data[f"{name}_eps"] = np.array(eps)
        data[f"{name}_min_samples"] = np.array(ms)
        data[f"{name}_labels"] = labels.astype(np.int32)
        data[f"{name}_centres"] = np.array(centres, dtype=np.float64).reshape(-1, 2)
        names.append(name)
    # update_known_landmarks over particles' maps (landmark_utils.py:120-144)
    N, L = 60, 25
    base = rng.uniform(-10, 10, (L, 2))
    parts, lm, cnt = [], np.zeros((N, L + 3, 6)), np.zeros(N, np.int32)
    for i in range(N):
        p = Particle(0.0, 0.0, 0.0)
        k = L + int(rng.integers(0, 4))
        xy = np.concatenate([base, rng.uniform(-10, 10, (k - L, 2))]) + rng.normal(0, 0.02, (k, 2))
        p.landmarks = [Landmark(float(x), float(y)) for x, y in xy]
        parts.append(p)
        cnt[i] = k
        lm[i, :k, 0:2] = xy
        lm[i, :k, 2] = lm[i, :k, 5] = 0.1
    LandmarkUtils.known_landmarks = []
    LandmarkUtils.update_known_landmarks(parts)
    data["known_lm"] = lm
    data["known_cnt"] = cnt
    data["known_centres"] = np.array([[k.x, k.y] for k in LandmarkUtils.known_landmarks]).reshape(-1, 2)
    data["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "cluster_cases.npz"), **data)
    print("wrote cluster_cases.npz:", names, "known centres", len(data["known_centres"]))


if __name__ == "__main__":
    main()
