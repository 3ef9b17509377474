"""Resamples whose sources take thousands of outputs (fast_slam_2.py:177-199):
a wave of k_ranges with more than kWaveFill outputs lists its sources' runs in
pieces for k_fill_runs (every workgroup takes pieces) instead of filling 64
outputs per step.  Three shapes, each one scan without measurements (the weights
are the imported ones) against the C oracle on the same draws: heavy particles --
two of them adjacent in one wave, one further on; a family of 128 heavy siblings
side by side (two waves of sources with ~156 outputs each); and normalised weights
that sum below 1 (total < 1, Q6), where the reference's
`min(particle_index + 1, N - 1)` hands every output past the total to the last
particle (Q10).  Every particle's state after the resample must be the oracle's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-9


def _weights(kind, N):
    w = np.full(N, 1e-9)
    if kind == "heavy":
        w[5], w[6], w[15000] = 0.3, 0.3, 0.2          # 7.5 K, 7.5 K and 5 K outputs
    elif kind == "family":                            # 128 heavy siblings side by side: ~156 outputs
        w[64:192] = 1.0 / 128                         # each, ~10 K per wave (listed in pieces)
    else:                                             # "short_total": sum of w' ~ 0.19
        w[:] = 0.09 / N
        w[1234] = 0.01
    return w


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind", ["heavy", "family", "short_total"])
@pytest.mark.parametrize("reduce", ["auto", "parallel"])
def test_long_output_runs_match_oracle(kind, reduce):
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    from oracle import oracle as orc
    configure()
    N, L = 20011, 16
    wl = syn.Workload(N, L, seed=11)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    w = _weights(kind, N)
    f = fast_slam_2.FastSLAM2(N, reduce=reduce, record_assoc=True, landmark_capacity=L + 8, verbose=False)
    f.set_state(x, y, yaw, w, np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, L + 8)
    o.set_state(x, y, yaw, w, np.full(N, L), lm)
    rng = np.random.default_rng(5)
    nz = rng.normal(0, 0.0055, N)
    u0 = rng.uniform(0, 1.0 / N)
    pose, st = f.step(0.0, 0.03, np.zeros((0, 2)), None, nz, u0)
    opose, _, ors, one = o.iterate(0.0, 0.03, np.zeros((0, 2)), nz, u0)
    assert ors and st.resampled
    assert np.isclose(st.n_eff, one, rtol=1e-12)
    assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12)
    xg, yg, yawg, wg, cg, lmg = f.get_state(lm_cap=L + 8)
    for a, b in ((xg, o.x), (yg, o.y), (yawg, o.yaw), (wg, o.w)):
        assert np.array_equal(a, b) or np.allclose(a, b, rtol=RTOL, atol=1e-15)
    assert np.array_equal(cg, o.cnt)
    assert np.allclose(lmg, o.lm, rtol=RTOL, atol=1e-12)
    # the outputs really were concentrated: a source fills a long run
    _, counts = np.unique(xg, return_counts=True)
    assert counts.max() >= 150
    f.close()
