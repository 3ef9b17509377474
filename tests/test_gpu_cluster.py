"""Known-landmark clustering on the GPU (fs2_cluster.hip; reference
GeometryUtils.cluster_points geometry_utils.py:26-62 and
LandmarkUtils.update_known_landmarks landmark_utils.py:120-144): labels equal to
sklearn's, centres bit-identical to the reference's numpy means."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _load():
    return np.load(os.path.join(GOLDEN, "cluster_cases.npz"))


def test_cluster_points_golden():
    from fast_slam_2 import GeometryUtils
    d = _load()
    for n in d["names"]:
        pts = d[f"{n}_points"]
        cen, lab = GeometryUtils.dbscan(pts, float(d[f"{n}_eps"]), int(d[f"{n}_min_samples"]))
        assert np.array_equal(lab, d[f"{n}_labels"]), n
        assert np.array_equal(cen, d[f"{n}_centres"]), n
        ref = GeometryUtils.cluster_points([tuple(p) for p in pts], float(d[f"{n}_eps"]),
                                           int(d[f"{n}_min_samples"]))
        assert len(ref) == len(cen) and all(np.array_equal(a, b) for a, b in zip(ref, cen))


def test_update_known_landmarks_golden():
    import fast_slam_2
    from fast_slam_2 import LandmarkUtils, Landmark, Particle
    from gpu_util import configure
    configure()
    d = _load()
    lm, cnt = d["known_lm"], d["known_cnt"]
    N = len(cnt)
    f = fast_slam_2.FastSLAM2(N, verbose=False, landmark_capacity=lm.shape[1])
    f.set_state(np.zeros(N), np.zeros(N), np.zeros(N), np.full(N, 1.0 / N), cnt, lm)
    LandmarkUtils.known_landmarks = []
    LandmarkUtils.update_known_landmarks(f.particles)          # device path
    got = np.array([[k.x, k.y] for k in LandmarkUtils.known_landmarks])
    assert np.array_equal(got, d["known_centres"])
    # host path over plain Particle objects gives the same
    parts = []
    for i in range(N):
        p = Particle(0.0, 0.0, 0.0)
        p.landmarks = [Landmark(float(lm[i, j, 0]), float(lm[i, j, 1])) for j in range(cnt[i])]
        parts.append(p)
    LandmarkUtils.known_landmarks = []
    LandmarkUtils.update_known_landmarks(parts)
    got2 = np.array([[k.x, k.y] for k in LandmarkUtils.known_landmarks])
    assert np.array_equal(got2, d["known_centres"])
    f.close()


def test_cluster_points_vs_sklearn_random():
    """Larger random sets with clusters of every density, against sklearn run here."""
    sk = pytest.importorskip("sklearn.cluster")
    from fast_slam_2 import GeometryUtils
    rng = np.random.default_rng(9)
    for trial in range(4):
        k = int(rng.integers(5, 40))
        centres = rng.uniform(-20, 20, (k, 2))
        sizes = rng.integers(5, 800, k)
        spread = rng.uniform(0.02, 0.4, k)
        pts = np.concatenate([rng.normal(c, s, (m, 2)) for c, s, m in zip(centres, spread, sizes)] +
                             [rng.uniform(-22, 22, (int(rng.integers(100, 3000)), 2))])
        pts = pts[rng.permutation(len(pts))]
        ms = int(rng.integers(3, 40))
        lab_ref = sk.DBSCAN(eps=0.5, min_samples=ms).fit(pts).labels_
        cen, lab = GeometryUtils.dbscan(pts, 0.5, ms)
        assert np.array_equal(lab, lab_ref), trial
        for rep in range(4):      # the union-find is concurrent: results must not vary
            assert np.array_equal(GeometryUtils.dbscan(pts, 0.5, ms)[1], lab_ref), (trial, rep)
        K = lab_ref.max() + 1
        for c in range(K):
            m = pts[lab_ref == c]
            assert np.array_equal(cen[c], m.mean(axis=0)), (trial, c)


def test_cluster_bad_input():
    from fast_slam_2 import GeometryUtils
    with pytest.raises(ValueError):
        GeometryUtils.dbscan(np.array([[0.0, np.nan], [1.0, 1.0]]), 0.5, 1)
    with pytest.raises(ValueError):
        GeometryUtils.dbscan(np.zeros((0, 2)), 0.5, 1)


def test_serializer_from_device_view():
    """Serializer given FastSLAM2.particles (one device download) writes the same text
    as the reference's per-object json.dump."""
    import json
    import fast_slam_2
    from fast_slam_2 import DirectedPoint, EvaluationResults, Point, Serializer
    from gpu_util import configure
    configure()
    N = 3000
    rng = np.random.default_rng(8)
    f = fast_slam_2.FastSLAM2(N, verbose=False)
    f.set_state(rng.normal(0, 3, N), rng.normal(0, 3, N), rng.uniform(-3, 3, N), np.full(N, 1.0 / N))
    est, act = DirectedPoint(0.5, 0.25, 0.1), DirectedPoint(0.0, 0.0, 0.0)
    lms = [Point(1.0, 2.0)]
    res = EvaluationResults("t", 0.0, 0.0, 0.0, 0.0, 0.0)
    x, y, yaw, *_ = f.get_state()
    want = json.dumps({"estimated_robot_pos": est.to_dict(), "actual_robot_pos": act.to_dict(),
                       "particles": [{"x": float(a), "y": float(b), "yaw": float(c)}
                                     for a, b, c in zip(x, y, yaw)],
                       "landmarks": [lm.to_dict() for lm in lms], "results": res.to_dict()}, indent=4)
    assert Serializer.to_json(est, act, f.particles, lms, res) == want
    assert len(f.particles) == N and f.particles[N - 1].yaw == yaw[N - 1]
    f.close()
