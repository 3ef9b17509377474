"""numpy's legacy RandomState drawn on the GPU (fs2_mt_draw), the drop-in
iterate()'s replacement for the reference's host draws
np.random.normal(0, ROTATION_NOISE / TRANSLATION_NOISE) per particle
(fast_slam_2/algorithms/fast_slam_2.py:79,81) and np.random.uniform(0, 1/N)
(:183).  numpy itself is the oracle: the device noise buffer, u0 and the state
after the normals / after u0 must equal what np.random produces from the same
state, bit for bit, at sizes from 1 to 4M particles, from states with a cached
gauss and with pos anywhere in the 624-word block (624 included), over
consecutive draws (the words of the next draw are made ahead on a side stream;
continuing after the normals or after u0 uses them, a reseed does not), drawn
synchronously (fs2_mt_draw) or deferred (fs2_mt_draw_deferred, ended by the
next call that needs it)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fs():
    import torch  # noqa: F401
    import fast_slam_2
    yield fast_slam_2


def draw(f, sigma, deferred=False):
    from fast_slam_2 import _native as nat
    lib = nat.load()
    st = np.random.get_state()
    mi, ma, mu, u0 = nat.fs2_mt_state.from_numpy(st), nat.fs2_mt_state(), nat.fs2_mt_state(), C.c_double()
    fn = lib.fs2_mt_draw_deferred if deferred else lib.fs2_mt_draw
    nat.check(fn(f._h, C.byref(mi), sigma, C.byref(ma), C.byref(mu), C.byref(u0)), f._h)
    out = np.empty(f.n_local)
    nat.check(lib.fs2_debug_noise(f._h, nat.ptr(out)), f._h)     # (ends a deferred draw)
    return st, out, ma.to_numpy(), mu.to_numpy(), u0.value


def same_state(a, b):
    return (a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]
            and a[4] == b[4])


@pytest.mark.parametrize("N,pre,words", [(1, 0, 0), (1, 1, 0), (2, 1, 3), (7, 0, 312), (1000, 0, 2),
                                         (1001, 3, 311), (65537, 1, 100), (1000000, 0, 0),
                                         (1000000, 1, 312), (4194304, 0, 7)])
def test_mt_draw_matches_numpy(fs, N, pre, words):
    np.random.seed(1000 * pre + words + N % 997)
    np.random.normal(size=pre)               # pre odd: a cached gauss
    np.random.random_sample(words)           # two words each: pos anywhere, 624 included
    f = fs.FastSLAM2(N, rng="numpy", verbose=False, landmark_capacity=8)
    for k, sigma in enumerate((0.0055, 0.001, 0.0055, 0.001)):
        if k == 3:
            np.random.seed(N + 7)            # the caller moves numpy elsewhere: words made ahead are not used
            np.random.random_sample(words % 5)
        st, out, after, after_u0, u0 = draw(f, sigma, deferred=(k % 2 == 1))
        np.random.set_state(st)
        ref = np.random.normal(0, sigma, size=N)
        bad = np.flatnonzero(out != ref)
        assert len(bad) == 0, (N, k, len(bad), bad[:5], out[bad[:5]], ref[bad[:5]])
        assert same_state(np.random.get_state(), after), (N, k)
        ru = np.random.uniform(0, 1 / N)
        assert ru == u0, (N, k, ru, u0)
        assert same_state(np.random.get_state(), after_u0), (N, k)
        # the next scan continues after the normals, or after u0 (a resample)
        np.random.set_state(after if k % 2 == 0 else after_u0)
    f.close()


def run_scans(fs, rng, N, L, scans, interfere=(), reseed_at=()):
    """The bench's synthetic state, `scans` iterate() calls from seed 17; on the scans
    in `interfere` the caller draws from numpy first, on those in `reseed_at` it
    reseeds.  Returns the per-scan outputs and numpy's final state."""
    import bench
    import fs2_synthetic as syn
    f = fs.FastSLAM2(N, rng=rng, verbose=False, landmark_capacity=L + scans + 8)
    bench.populate(f, N, L, 3, 0)              # the bench's synthetic state (seeded, identical)
    np.random.seed(17)
    out = []
    for s in range(scans):
        if s in interfere:
            np.random.random_sample(3)
        if s in reseed_at:
            np.random.seed(100 + s)
        rot, tr = syn.odometry(s)
        ms = [fs.Measurement(float(d), float(b)) for d, b in syn.scan_measurements(L, s, 3)]
        pose = f.iterate(rot, tr, ms)
        st = f.last_stats
        out.append((pose, st.resampled, st.n_eff, f.get_state(lm_cap=L + scans + 8)))
    f.close()
    return out, np.random.get_state()


def assert_same_runs(a, b):
    assert same_state(a[1], b[1])
    assert sum(o[1] for o in a[0]) >= 1
    for s, (oa, ob) in enumerate(zip(a[0], b[0])):
        assert oa[0] == ob[0] and oa[1] == ob[1] and oa[2] == ob[2], s
        for u, v in zip(oa[3], ob[3]):
            assert np.array_equal(u, v), s


def test_iterate_device_draws_equal_host_draws(fs):
    """Two handles from the same state, one drawing numpy's stream on the GPU, one
    with numpy on the host: every scan's pose, decision, state and numpy's state
    afterwards agree bit for bit (resampling scans included; the odometry
    alternates the two noise scales)."""
    from gpu_util import configure
    configure()
    N, L, scans = 20000, 40, 8
    a = run_scans(fs, "numpy", N, L, scans)
    b = run_scans(fs, "numpy-host", N, L, scans)
    assert_same_runs(a, b)


def test_draw_follows_numpy_when_the_caller_moves_it(fs):
    """The caller draws from numpy (scans 2, 5) or reseeds it (scan 4) between
    iterate() calls: every draw starts from numpy's actual state -- bit for bit the
    host draws."""
    from gpu_util import configure
    configure()
    N, L, scans = 20000, 40, 7
    kw = dict(interfere=(2, 5), reseed_at=(4,))
    a = run_scans(fs, "numpy", N, L, scans, **kw)
    b = run_scans(fs, "numpy-host", N, L, scans, **kw)
    assert_same_runs(a, b)


def test_mt_draw_rejects_negative_scale(fs):
    """numpy's normal raises ValueError for scale < 0; so does the device draw."""
    from fast_slam_2 import _native as nat
    lib = nat.load()
    f = fs.FastSLAM2(64, rng="numpy", verbose=False, landmark_capacity=8)
    mi = nat.fs2_mt_state.from_numpy(np.random.get_state())
    ma, mu = nat.fs2_mt_state(), nat.fs2_mt_state()
    for bad in (-1e-3, float("nan")):
        with pytest.raises(ValueError):
            nat.check(lib.fs2_mt_draw(f._h, C.byref(mi), bad, C.byref(ma), C.byref(mu), None), f._h)
    f.close()


def test_deferred_draw_ends_on_every_path(fs):
    """A deferred draw writes its outputs whatever ends it: a scan that rejects
    explicit noise after it (FS2_ERR_ARG), or a state write; the handle works on."""
    from fast_slam_2 import _native as nat
    lib = nat.load()
    N = 4096
    f = fs.FastSLAM2(N, rng="numpy", verbose=False, landmark_capacity=8)
    np.random.seed(5)
    st = np.random.get_state()
    ref = np.random.normal(0, 0.001, size=N)
    after_ref = np.random.get_state()
    for end in ("submit", "set_state"):
        mi, ma, mu = nat.fs2_mt_state.from_numpy(st), nat.fs2_mt_state(), nat.fs2_mt_state()
        nat.check(lib.fs2_mt_draw_deferred(f._h, C.byref(mi), 0.001, C.byref(ma), C.byref(mu), None), f._h)
        if end == "submit":
            nz = np.zeros(N)
            rc = lib.fs2_iterate_submit(f._h, 0.0, 0.1, None, None, 0, nat.ptr(nz), None)
            assert rc == nat.FS2_ERR_ARG
        else:
            x, y, yaw, w, c, lm = f.get_state(lm_cap=8)
            f.set_state(x, y, yaw, w, c, lm)
        assert same_state(ma.to_numpy(), after_ref), end
        out = np.empty(N)
        nat.check(lib.fs2_debug_noise(f._h, nat.ptr(out)), f._h)
        assert np.array_equal(out, ref), end
    f.close()


def test_full_size_dropin_device_draws_equal_host_draws(fs):
    """BASELINE config 3 (10^6 particles, L = 500, the bench's synthetic state and
    stream) through iterate(): numpy's stream drawn on the GPU (deferred: ended
    beside the candidate pass) against numpy drawing on the host.  Every scan's pose, decision, N_eff and total weight are equal, so
    are every particle's pose and weight after the run and numpy's final state."""
    import bench
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()                      # config.py's defaults (earlier tests may change them)
    N, L, scans = 1_000_000, 500, 6
    out = {}
    for rng in ("numpy", "numpy-host"):
        np.random.seed(3)
        f = fs.FastSLAM2(N, rng=rng, seed=0, landmark_capacity=L + scans + 8, verbose=False)
        bench.populate(f, N, L, 0, 0)
        per = []
        for s in range(scans):
            ms = [fs.Measurement(float(d), float(b)) for d, b in syn.scan_measurements(L, s, 0)]
            pose = f.iterate(*syn.odometry(s), ms)
            st = f.last_stats
            per.append((pose, st.resampled, st.n_eff, st.total_weight))
        x, y, yaw, w, cnt, _ = f.get_state(lm_cap=0)
        f.close()
        out[rng] = (per, (x, y, yaw, w, cnt), np.random.get_state())
    a, b = out["numpy"], out["numpy-host"]
    assert a[0] == b[0]
    assert sum(p[1] for p in a[0]) >= 1
    for u, v in zip(a[1], b[1]):
        assert np.array_equal(u, v)
    assert same_state(a[2], b[2])
