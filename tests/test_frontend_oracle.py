"""The front-end oracle (oracle/fs2_frontend_oracle.c) against the reference's
own outputs (tests/golden/frontend_cases.npz, made by gen_frontend.py) and
against numpy's float32 trigonometry.  CPU only."""
import os

import numpy as np
import pytest

from oracle import oracle as orc

GOLD = os.path.join(os.path.dirname(__file__), "golden", "frontend_cases.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_numpy_float32_sincos_restatement():
    th = np.float32(np.pi / 180)
    grid = (np.arange(180).astype(np.float32) * th).astype(np.float32)
    rnd = np.random.default_rng(3).uniform(-50.0, 50.0, 20000).astype(np.float32)
    for x in np.concatenate([grid, rnd, np.float32([0.0, -0.0, np.pi, -np.pi, 1e-30])]):
        assert orc.np_sinf(x) == np.sin(x), x
        assert orc.np_cosf(x) == np.cos(x), x


def _scenes(gold):
    return [str(s) for s in gold["scenes"]]


def test_image_geometry_and_raster(gold):
    for s in _scenes(gold):
        pts = gold[f"{s}/points"]
        filt = orc.line_filter(pts)
        img, g = orc.fe_image(filt)
        w, h = gold[f"{s}/wh"]
        assert (g[2], g[3]) == (w, h), s
        ref = np.zeros((h, w), np.uint8)
        for x, y in gold[f"{s}/circle_centres"]:
            for dy, hw in zip(range(-2, 3), (0, 1, 2, 1, 0)):
                ref[y + dy, x - hw:x + hw + 1] = 255
        assert np.array_equal(img, ref), s


def test_intersections_clusters_corners_measurements(gold):
    n_meas = 0
    for s in _scenes(gold):
        pts = gold[f"{s}/points"]
        filt = orc.line_filter(pts)
        _, g = orc.fe_image(filt)
        lines = gold[f"{s}/lines"]
        isf = orc.fe_intersections(lines, g[2], g[3])
        ip = orc.fe_back(isf, g[0], g[1])
        assert np.array_equal(ip, gold[f"{s}/intersections"]), s
        cent = orc.fe_cluster1(ip) if len(ip) else np.zeros((0, 2))
        assert np.array_equal(cent, gold[f"{s}/clusters"]), s
        corners = orc.fe_corners(cent, filt)
        assert np.array_equal(corners, gold[f"{s}/corners"]), s
        meas = orc.fe_measure(corners)
        assert np.array_equal(meas, gold[f"{s}/measurements"]), s
        m, counts = orc.fe_extract(pts)
        assert np.array_equal(m, gold[f"{s}/measurements"]), s
        assert list(counts) == [len(lines), len(ip), len(cent), len(corners)], s
        n_meas += len(m)
    assert n_meas > 30


def test_intersection_algebra_random_sets(gold):
    for k in range(int(gold["isect_sets"])):
        lines = gold[f"isect/{k}/lines"]
        w, h = gold[f"isect/{k}/wh"]
        out = orc.fe_intersections(lines, int(w), int(h)).astype(np.float64)
        assert np.array_equal(out, gold[f"isect/{k}/out"]), k


def test_legacy_promotion_close_to_nep50(gold):
    """numpy 1.x promotion (float64 after the back-conversion) stays within
    float32 rounding of the pinned NEP 50 results."""
    for s in _scenes(gold):
        m, _ = orc.fe_extract(gold[f"{s}/points"], legacy=True)
        ref = gold[f"{s}/measurements"]
        assert m.shape == ref.shape, s
        assert np.allclose(m, ref, rtol=1e-6, atol=1e-6), s
