"""Pin the CPU oracle against golden vectors recorded from the reference.

The fixtures under tests/golden/ were produced by tests/golden/gen_golden.py,
which runs the reference (cy-rae/fast-slam) itself in the build container.
Bars: association indices and resample sources bit-exact; the Mahalanobis
gate distance bit-exact (OpenBLAS FMA order restated); poses, landmark means,
covariances and weights within 1e-9 relative per scan sequence (ulp-level
differences from numpy's SIMD atan2/exp and scipy's eigh-based pdf).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as orc

SEQS = sorted(f[4:-4] for f in os.listdir(GOLDEN) if f.startswith("seq_") and f.endswith(".npz"))


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def close(a, b, rtol=1e-9, atol=1e-12):
    return np.allclose(a, b, rtol=rtol, atol=atol)


def test_pymod_matches_numpy_remainder():
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.normal(0, 10, 5000), [0.0, -0.0, np.pi, -np.pi, 2 * np.pi, 1e-300]])
    two_pi = 2 * np.pi
    for v in vals:
        assert orc.pymod(v, two_pi) == (np.float64(v) % two_pi)


def test_inv2_bit_exact_vs_numpy():
    rng = np.random.default_rng(1)
    for _ in range(3000):
        A = rng.normal(0, 1, (2, 2))
        A = A @ A.T + 0.01 * np.eye(2)
        A[0, 1] += rng.normal(0, 1e-3)
        assert np.array_equal(orc.inv2(A), np.linalg.inv(A))
    with pytest.raises(np.linalg.LinAlgError):
        orc.inv2(np.zeros((2, 2)))


def test_np_sum_order():
    rng = np.random.default_rng(2)
    for n in [1, 2, 7, 8, 9, 127, 128, 129, 1000, 8191, 8192, 8193, 20000, 100003]:
        a = rng.random(n) ** 3
        assert orc.np_sum(a) == np.sum(a), n


def test_mahalanobis_and_association_golden():
    d = load("unit_geometry.npz")
    for k in range(len(d["a"])):
        got = orc.mahalanobis(d["a"][k], d["b"][k], d["cov"][k])
        assert got == d["dist"][k], k
    for q in range(len(d["observed"])):
        lm = np.concatenate([d["lm"][q], d["lm_cov"][q].reshape(-1, 4)], axis=1)
        assert orc.associate(d["observed"][q], lm, float(d["gate"])) == d["assoc"][q], q


def test_weights_golden():
    d = load("unit_weights.npz")
    for k in range(int(d["count"])):
        w = d[f"w{k}"]
        wn = orc.normalize(w)
        assert np.array_equal(wn, d[f"wn{k}"]), k
        assert orc.n_eff(wn) == d["n_eff"][k], k
        src = orc.resample_src(wn, d["u0"][k])
        if d[f"src{k}"][0] >= 0:
            assert np.array_equal(src, d[f"src{k}"]), k
            # estimate = first max over the resampled weights, reported as old index
            assert src[orc.argmax_first(wn[src])] == d["est_index"][k]


def test_resample_no_hang_rule():
    # weights sum < 1 with a zero last weight: the reference loops forever (Q10)
    w = np.array([0.3, 0.3, 0.3, 0.0])
    src = orc.resample_src(w, 0.249)
    assert src.tolist() == [0, 1, 2, 3]


def test_line_filter_golden():
    d = load("unit_linefilter.npz")
    for k, s in enumerate(d["sigma"]):
        assert np.allclose(orc.line_filter(d["points"], s), d["out"][k], rtol=1e-14, atol=1e-14)
        assert np.allclose(orc.line_filter(d["short"], s), d["out_short"][k], rtol=1e-14,
                           atol=1e-14)
    assert np.array_equal(orc.line_filter(d["points"], 0.1), d["points"])   # Q13


def test_best_fit_golden():
    d = load("unit_bft.npz")
    for k in range(len(d["src"])):
        R, t = orc.best_fit(d["src"][k], d["tgt"][k])
        assert np.allclose(R, d["R"][k], atol=1e-13)
        assert np.allclose(t, d["t"][k], atol=1e-12)


def test_icp_golden():
    d = load("unit_icp.npz")
    k180 = k720 = 0
    for k, P in enumerate(d["P"]):
        if P == 180:
            src, tgt = d["src180"][k180], d["tgt180"][k180]
            k180 += 1
        else:
            src, tgt = d["src720"][k720], d["tgt720"][k720]
            k720 += 1
        R, t, it = orc.icp(src, tgt)
        assert it == d["iters"][k], (k, it, d["iters"][k])
        assert np.allclose(R, d["R"][k], atol=1e-10)
        assert np.allclose(t, d["t"][k], atol=1e-10)


@pytest.mark.parametrize("name", SEQS)
def test_sequence_golden(name):
    d = load(f"seq_{name}.npz")
    N, S, cap = int(d["N"]), int(d["S"]), int(d["cap"])
    tr, rot, mn = d["noise_cfg"]
    f = orc.OracleFilter(N, cap, tr_noise=tr, rot_noise=rot, meas_noise=np.eye(2) * mn,
                         gate=float(d["gate"]))
    f.set_state(d["x"][0], d["y"][0], d["yaw"][0], d["w"][0], d["cnt"][0], d["lm"][0])
    for s in range(S):
        M = int(d["M"][s])
        u0 = d["uniform"][s]
        pose, assoc, rs, ne = f.iterate(d["rotation"][s], d["translation"][s], d["meas"][s, :M],
                                        d["normals"][s], 0.0 if np.isnan(u0) else u0,
                                        observed=d["observed"][s, :M])
        assert np.array_equal(assoc, d["assoc"][s, :M]), (name, s)
        assert rs == (not np.isnan(u0)), (name, s)
        assert np.isclose(ne, d["n_eff"][s], rtol=1e-9), (name, s)
        assert close(pose, d["estimate"][s]), (name, s)
        assert np.array_equal(f.cnt, d["cnt"][s + 1]), (name, s)
        assert close(f.x, d["x"][s + 1]) and close(f.y, d["y"][s + 1]), (name, s)
        assert close(f.yaw, d["yaw"][s + 1]), (name, s)
        assert close(f.w, d["w"][s + 1], rtol=1e-8), (name, s)
        k = min(cap, d["lm"].shape[2])
        assert close(f.lm[:, :k], d["lm"][s + 1][:, :k], rtol=1e-8, atol=1e-12), (name, s)
