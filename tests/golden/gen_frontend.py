#!/usr/bin/env python3
"""Golden fixtures for the landmark front-end.

Runs the reference's own LandmarkUtils.get_measurements_to_landmarks /
get_observed_landmarks (fast_slam_2/utils/landmark_utils.py:21-89) and
HoughTransformation (fast_slam_2/algorithms/hough_transformation.py:14-145)
in this container and records their outputs.  opencv-python is not installed,
so the `cv2` module the reference imports is a stub here:

  * cv2.circle records the centre the reference computes and draws OpenCV's
    filled radius-2 circle (a 13-pixel diamond) into the reference's image;
  * cv2.HoughLines records the image and threshold and returns the lines of
    the C oracle's restatement of OpenCV's HoughLinesStandard.

Everything else -- image geometry, intersections (numpy float32 scalar
arithmetic), back-conversion, sklearn DBSCAN + numpy means, the corner test
and the (distance, angle) conversion -- is the reference's code, so those
stages are pinned; the raster and the Hough vote are pinned only to the
published OpenCV algorithm (parity unpinned against OpenCV itself).

Also records the reference's private __calculate_intersections on random line
sets (theta on OpenCV's n * (float)(pi/180) grid) to pin the float32 algebra.

Run:  python tests/golden/gen_frontend.py   (writes tests/golden/frontend_cases.npz)
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [REPO, os.path.join(REPO, "fast-slam_amd")]

import fs2_synthetic as syn  # noqa: E402
from oracle import oracle as orc  # noqa: E402

REC = {"centres": [], "images": [], "thresholds": []}
HALF = (0, 1, 2, 1, 0)


def _circle(image, center, radius, color, thickness):
    assert radius == 2 and thickness == -1
    x, y = int(center[0]), int(center[1])
    REC["centres"].append((x, y))
    for dy in range(-2, 3):
        h = HALF[dy + 2]
        image[y + dy, x - h:x + h + 1] = color
    return image


def _hough(image, rho, theta, threshold):
    assert rho == 1 and theta == np.pi / 180
    REC["images"].append(image.shape)
    REC["thresholds"].append(threshold)
    lines = orc.fe_hough(image, threshold)
    return lines.reshape(-1, 1, 2) if len(lines) else None


def import_reference():
    cv2 = types.ModuleType("cv2")
    cv2.circle = _circle
    cv2.HoughLines = _hough
    sys.modules["cv2"] = cv2
    sys.modules.setdefault("HAL", types.ModuleType("HAL"))
    sys.path.insert(0, REF)
    from fast_slam_2.algorithms.hough_transformation import HoughTransformation
    from fast_slam_2.algorithms.line_filter import LineFilter
    from fast_slam_2.utils.geometry_utils import GeometryUtils
    from fast_slam_2.utils.landmark_utils import LandmarkUtils
    return HoughTransformation, LineFilter, GeometryUtils, LandmarkUtils


def scenes(rng):
    out = []
    poses = [(0.0, 0.0, 0.3), (-3.0, 2.0, -1.0), (1.0, -2.0, 2.2), (-4.5, -3.0, 0.7), (0.5, 3.5, -2.5)]
    for P in (180, 360, 720):
        for k, pose in enumerate(poses):
            out.append((f"lroom_P{P}_{k}", syn.polygon_scan(syn.L_ROOM, pose, P, rng)))
    for k, pose in enumerate([(0.0, 0.0, 0.0), (6.0, 4.0, 0.6), (-7.0, -5.0, -2.4)]):
        out.append((f"box_{k}", syn.polygon_scan(syn.BOX_ROOM, pose, 180, rng, max_range=30.0)))
    # no corner in view / a single wall / a wall corner only
    out.append(("wall", syn.polygon_scan(syn.BOX_ROOM, (0.0, 0.0, 0.0), 180, rng, max_range=8.0)))
    out.append(("far_noise", syn.polygon_scan(syn.L_ROOM, (0.0, 0.0, 0.3), 180, rng, noise=0.05)))
    out.append(("tiny", syn.polygon_scan(syn.L_ROOM, (5.0, -3.0, 0.8), 180, rng, max_range=1.5)))
    out.append(("positive_min", syn.polygon_scan(syn.L_ROOM, (-5.9, -3.9, 0.8), 180, rng)))
    return out


def main():
    Hough, LineFilter, GeometryUtils, LandmarkUtils = import_reference()
    rng = np.random.default_rng(20250103)
    data = {"numpy": np.__version__}
    import sklearn
    data["sklearn"] = sklearn.__version__
    names = []
    for name, pts in scenes(rng):
        names.append(name)
        REC["centres"].clear()
        REC["images"].clear()
        meas = LandmarkUtils.get_measurements_to_landmarks(pts)
        lms = LandmarkUtils.get_observed_landmarks(pts)
        filt = LineFilter.filter(pts)
        isect = Hough.detect_line_intersections(filt)
        cent = GeometryUtils.cluster_points(isect, 0.5, 1) if len(isect) else []
        h, w = REC["images"][0]
        lines = orc.fe_hough(orc.fe_image(filt)[0])
        data[f"{name}/points"] = pts
        data[f"{name}/wh"] = np.array([w, h], np.int64)
        data[f"{name}/circle_centres"] = np.array(REC["centres"][:len(pts)], np.int64).reshape(-1, 2)
        data[f"{name}/lines"] = lines.reshape(-1, 2)
        data[f"{name}/intersections"] = np.array([[float(x), float(y)] for x, y in isect]).reshape(-1, 2)
        data[f"{name}/intersection_f32"] = np.array(
            [isinstance(x, np.float32) for x, _ in isect] or [True], bool)
        data[f"{name}/clusters"] = np.array([[float(c[0]), float(c[1])] for c in cent]).reshape(-1, 2)
        data[f"{name}/corners"] = np.array([[float(l.x), float(l.y)] for l in lms]).reshape(-1, 2)
        data[f"{name}/measurements"] = np.array([[m.distance, m.yaw] for m in meas]).reshape(-1, 2)
        print(f"{name}: {len(pts)} pts, {len(lines)} lines, {len(isect)} intersections, "
              f"{len(cent)} clusters, {len(meas)} measurements")
    data["scenes"] = np.array(names)

    # the float32 intersection algebra on random line sets
    calc = Hough._HoughTransformation__calculate_intersections
    th = np.float32(np.pi / 180)
    sets = []
    for k in range(40):
        K = int(rng.integers(2, 40))
        n = rng.integers(0, 180, K)
        theta = (np.float32(0.0) + n.astype(np.float32) * th).astype(np.float32)
        rho = (rng.integers(-3000, 3000, K).astype(np.float32) + np.float32(0.5) * rng.integers(0, 2, K)
               ).astype(np.float32)
        lines = np.stack([rho, theta], axis=1).astype(np.float32).reshape(-1, 1, 2)
        w, h = int(rng.integers(200, 3000)), int(rng.integers(200, 3000))
        res = calc(lines, w, h)
        sets.append((lines.reshape(-1, 2), w, h, np.array([[float(x), float(y)] for x, y in res]).reshape(-1, 2)))
    data["isect_sets"] = np.array(len(sets))
    for k, (lines, w, h, res) in enumerate(sets):
        data[f"isect/{k}/lines"] = lines
        data[f"isect/{k}/wh"] = np.array([w, h], np.int64)
        data[f"isect/{k}/out"] = res
    np.savez_compressed(os.path.join(HERE, "frontend_cases.npz"), **data)


if __name__ == "__main__":
    main()
