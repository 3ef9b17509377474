"""Known-landmark clustering fixtures (tests/golden/gen_cluster.py) pinned against
sklearn's DBSCAN in this environment (the library the reference calls in
geometry_utils.py:26-62): labels equal, and each recorded reference centre equals
the numpy mean of its cluster's points in index order."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _load():
    return np.load(os.path.join(GOLDEN, "cluster_cases.npz"))


def test_fixture_labels_match_sklearn():
    sk = pytest.importorskip("sklearn.cluster")
    d = _load()
    for n in d["names"]:
        pts = d[f"{n}_points"]
        lab = sk.DBSCAN(eps=float(d[f"{n}_eps"]), min_samples=int(d[f"{n}_min_samples"])).fit(pts).labels_
        assert np.array_equal(lab, d[f"{n}_labels"]), n


def test_fixture_centres_are_index_order_means():
    d = _load()
    for n in d["names"]:
        pts, lab, cen = d[f"{n}_points"], d[f"{n}_labels"], d[f"{n}_centres"]
        K = lab.max() + 1
        assert len(cen) == K, n
        for k in range(K):
            m = pts[lab == k]
            s = np.zeros(2)
            for p in m:                  # sequential, like numpy mean(axis=0)
                s = s + p
            assert np.array_equal(cen[k], s / len(m)), (n, k)
