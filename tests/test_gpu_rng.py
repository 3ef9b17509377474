"""The device generator behind rng="device" (every bench scan).

libfs2 replaces the reference's np.random draws -- one normal per particle per
scan for the motion sample (fast_slam_2.py:79,81) and the resample start u0
(:183) -- with counter-based Philox4x32-10 (fs2_device.hpp).  Pinned here:
  * Philox4x32-10 against the published Random123 known-answer vectors
    (kat_vectors: zero counter/key, all-ones, and the pi-digits case);
  * the Box-Muller normals' distribution over 1e7 draws: mean, variance,
    kurtosis, the 3- and 4-sigma tail masses, and a Kolmogorov-Smirnov test;
  * that the motion sample uses exactly those draws: particle g of scan s moves
    by sigma * normal(seed, s, g) (checked on the yaw of a rotation scan).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# Random123 kat_vectors, philox4x32 with 10 rounds: counter[4], key[2] -> output[4]
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def test_philox_known_answers():
    from fast_slam_2 import _native as nat
    lib = nat.load()
    ctr = np.array([c for c, _, _ in KAT], dtype=np.uint32)
    key = np.array([k for _, k, _ in KAT], dtype=np.uint32)
    out = np.zeros_like(ctr)
    nat.check(lib.fs2_debug_philox(0, len(KAT), ctr.ctypes.data, key.ctypes.data, out.ctypes.data))
    want = np.array([o for _, _, o in KAT], dtype=np.uint32)
    assert np.array_equal(out, want), [[hex(v) for v in r] for r in out]


def _normals(seed, stream, first, n):
    from fast_slam_2 import _native as nat
    lib = nat.load()
    out = np.empty(n)
    nat.check(lib.fs2_debug_normals(0, seed, stream, first, n, out.ctypes.data))
    return out


def test_normal_moments_and_tails():
    from scipy import stats
    n = 10_000_000
    z = _normals(0x5EEDF5A2, 7, 0, n)
    assert np.isfinite(z).all()
    se = 1.0 / np.sqrt(n)
    assert abs(z.mean()) < 5 * se
    assert abs(z.var() - 1.0) < 5 * np.sqrt(2.0) * se
    kurt = np.mean(z ** 4)
    assert abs(kurt - 3.0) < 5 * np.sqrt(96.0) * se          # var(z^4) = 105 - 9
    for k in (3.0, 4.0):
        p = 2 * stats.norm.sf(k)
        got = np.mean(np.abs(z) > k)
        assert abs(got - p) < 5 * np.sqrt(p * (1 - p) / n), (k, got, p)
    assert stats.kstest(z[:1_000_000], "norm").pvalue > 1e-4
    # different streams (scans) and seeds are different sequences
    assert not np.array_equal(z[:1000], _normals(0x5EEDF5A2, 8, 0, 1000))
    assert not np.array_equal(z[:1000], _normals(0x5EEDF5A3, 7, 0, 1000))
    assert np.array_equal(z[500:1500], _normals(0x5EEDF5A2, 7, 500, 1000))


def test_motion_sample_uses_the_device_normals():
    """A rotation scan without measurements: yaw' = pymod(yaw + rot + sigma z + pi, 2 pi) - pi
    (fast_slam_2.py:77-87) with z = normal(seed, scan, particle)."""
    import fast_slam_2
    from gpu_util import configure
    configure()
    N, seed = 5000, 1234
    f = fast_slam_2.FastSLAM2(N, rng="device", seed=seed, verbose=False)
    rng = np.random.default_rng(0)
    yaw0 = rng.uniform(-3, 3, N)
    f.set_state(np.zeros(N), np.zeros(N), yaw0, np.full(N, 1.0 / N))
    rot = 0.05
    f.step(0.0, 0.0, np.zeros((0, 2)))            # scan 0: translation noise only
    x, y, yaw1, _, _, _ = f.get_state()
    f.step(rot, 0.0, np.zeros((0, 2)))            # scan 1: rotation, yaw noise
    _, _, yaw2, _, _, _ = f.get_state()
    f.close()
    z1 = _normals(seed, 1, 0, N)
    want = np.mod(yaw1 + (rot + 0.001 * z1) + np.pi, 2 * np.pi) - np.pi
    assert np.allclose(yaw2, want, rtol=0, atol=1e-12)
    # scan 0 moved each particle by 0.0055 z0 along its (unchanged) heading
    z0 = _normals(seed, 0, 0, N)
    assert np.allclose(x, 0.0055 * z0 * np.cos(yaw1), rtol=0, atol=1e-12)
    assert np.allclose(y, 0.0055 * z0 * np.sin(yaw1), rtol=0, atol=1e-12)
