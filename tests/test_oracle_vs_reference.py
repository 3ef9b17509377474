"""Property tests: the C oracle against the reference itself on random inputs.

SURVEY.md §4's build test plan: per primitive, random cases (including edge
cases: ill-conditioned covariances, weights below the 1e-5 floor, zero weights,
exact ties, resample start points at cumulative-weight boundaries) are run
through the reference (tests/ref_primitives.py, in a subprocess because the
reference package is also named `fast_slam_2`) and through the oracle.  Runs in
the build container only; skipped where /root/reference is absent (the GPU box).

Bars: Mahalanobis distance, association index, normalised weights, N_eff,
estimate index and resample sources bit-exact; best-fit / ICP / LineFilter
within 1e-12 (SVD / KDTree / scipy correlate vs closed forms).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as orc

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "fast_slam_2")),
                                reason="reference not present (build container only)")


def _cases(rng):
    c = {}
    n = 1500
    a, b = rng.normal(0, 5, (n, 2)), rng.normal(0, 5, (n, 2))
    A = rng.normal(0, 1, (n, 2, 2))
    cov = A @ A.transpose(0, 2, 1) + 1e-3 * np.eye(2)
    cov[::7] *= 1e-6                                    # tiny / ill-conditioned
    cov[1::11, 0, 1] += rng.normal(0, 1e-2, len(cov[1::11]))   # slightly asymmetric
    c["maha_a"], c["maha_b"], c["maha_cov"] = a, b, cov
    K, Lmax = 300, 40
    lm = np.zeros((K, Lmax, 6))
    lens = rng.integers(0, Lmax + 1, K)
    obs = rng.normal(0, 3, (K, 2))
    for k in range(K):
        L = lens[k]
        lm[k, :L, 0:2] = obs[k] + rng.normal(0, 2.5, (L, 2))
        s = rng.uniform(0.01, 0.5, L)
        lm[k, :L, 2] = lm[k, :L, 5] = s
        lm[k, :L, 3] = lm[k, :L, 4] = rng.normal(0, 0.3, L) * s
    c["as_obs"], c["as_lm"], c["as_len"] = obs, lm, lens
    c["as_gate"] = rng.choice([8.0, 2.0, 0.5, 20.0], K)
    W, Nmax = 250, 64
    w = np.zeros((W, Nmax))
    wl = rng.integers(1, Nmax + 1, W)
    u0 = np.zeros(W)
    for k in range(W):
        N = wl[k]
        kind = k % 5
        if kind == 0:
            v = rng.random(N) ** 8
        elif kind == 1:
            v = np.where(rng.random(N) < 0.5, rng.random(N) * 1e-6, rng.random(N))   # below the floor
        elif kind == 2:
            v = np.zeros(N)
            v[rng.integers(0, N)] = rng.random()
        elif kind == 3:
            v = np.full(N, 1.0 / N)                                               # exact ties
        else:
            v = rng.random(N) * 1e-7                                              # total < 1e-5
        w[k, :N] = v
        nv = orc.normalize(v)
        cs = np.cumsum(nv)
        # u0 in (0, 1/N) or on a cumulative boundary reachable from it
        u0[k] = rng.uniform(0, 1.0 / N) if k % 3 else max(0.0, min(cs[0] % (1.0 / N), np.nextafter(1.0 / N, 0)))
    c["w"], c["w_len"], c["u0"] = w, wl, u0
    B, P = 60, 50
    src = rng.normal(0, 3, (B, P, 2))
    th = rng.uniform(-np.pi, np.pi, B)
    Rm = np.stack([np.stack([np.cos(th), -np.sin(th)], -1), np.stack([np.sin(th), np.cos(th)], -1)], -2)
    tgt = np.einsum("bij,bpj->bpi", Rm, src) + rng.normal(0, 2, (B, 1, 2)) + rng.normal(0, 0.01, (B, P, 2))
    c["bf_src"], c["bf_tgt"] = src, tgt
    I, Q = 12, 120
    base = rng.normal(0, 4, (I, Q, 2))
    ang = rng.uniform(-0.2, 0.2, I)
    Ri = np.stack([np.stack([np.cos(ang), -np.sin(ang)], -1), np.stack([np.sin(ang), np.cos(ang)], -1)], -2)
    c["icp_src"] = base
    c["icp_tgt"] = np.einsum("bij,bpj->bpi", Ri, base) + rng.normal(0, 0.3, (I, 1, 2))
    F = 40
    c["lf_pts"] = rng.normal(0, 3, (F, 90, 2))
    c["lf_sigma"] = rng.choice([0.1, 0.3, 0.5, 1.0, 2.5], F)
    return c


@pytest.fixture(scope="module")
def both(tmp_path_factory):
    rng = np.random.default_rng(20241015)
    cases = _cases(rng)
    d = tmp_path_factory.mktemp("ref")
    np.savez(d / "cases.npz", **cases)
    r = subprocess.run([sys.executable, os.path.join(HERE, "ref_primitives.py"), str(d / "cases.npz"),
                        str(d / "out.npz")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return cases, dict(np.load(d / "out.npz"))


def test_mahalanobis_bit_exact(both):
    c, r = both
    got = np.array([orc.mahalanobis(a, b, cv) for a, b, cv in zip(c["maha_a"], c["maha_b"], c["maha_cov"])])
    assert np.array_equal(got, r["maha"], equal_nan=True)


def test_association_exact(both):
    c, r = both
    for k in range(len(c["as_obs"])):
        L = c["as_len"][k]
        assert orc.associate(c["as_obs"][k], c["as_lm"][k, :L], c["as_gate"][k]) == r["assoc"][k], k


def test_weights_neff_estimate_resample(both):
    c, r = both
    hung = 0
    for k in range(len(c["w_len"])):
        N = c["w_len"][k]
        w = c["w"][k, :N]
        nw = orc.normalize(w)
        assert np.array_equal(nw, r["norm_w"][k, :N]), k
        assert orc.n_eff(nw) == r["n_eff"][k], k
        assert orc.argmax_first(nw) == int(r["est_x"][k]), k
        src = orc.resample_src(nw, c["u0"][k])
        if r["src"][k, 0] == -2:
            hung += 1                      # reference hangs (Q10); the oracle ends on N-1
            continue
        assert np.array_equal(src, r["src"][k, :N]), k
    assert hung < len(c["w_len"]) // 4


def test_best_fit_and_icp(both):
    c, r = both
    for k in range(len(c["bf_src"])):
        R, t = orc.best_fit(c["bf_src"][k], c["bf_tgt"][k])
        assert np.allclose(R, r["bf_R"][k], atol=1e-12) and np.allclose(t, r["bf_t"][k], atol=1e-11), k
    for k in range(len(c["icp_src"])):
        R, t, _ = orc.icp(c["icp_src"][k], c["icp_tgt"][k])
        assert np.allclose(R, r["icp_R"][k], atol=1e-10) and np.allclose(t, r["icp_t"][k], atol=1e-9), k


def test_line_filter(both):
    c, r = both
    for k in range(len(c["lf_pts"])):
        got = orc.line_filter(c["lf_pts"][k], c["lf_sigma"][k])
        assert np.allclose(got, r["lf"][k], rtol=1e-13, atol=1e-13), k
