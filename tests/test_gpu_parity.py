"""GPU parity: libfs2 (HIP, gfx950) against the reference's golden vectors and the
CPU oracle.  Every call goes through the C ABI (ctypes).

Bars: association indices and resample decisions bit-exact;
poses, landmark means/covariances and weights within 1e-5 (asserted much
tighter here: 1e-8 relative -- the only differences are ulp-level ones between
the device's fp64 libm (ocml) and glibc/numpy transcendentals).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

SEQS = sorted(f[4:-4] for f in os.listdir(GOLDEN) if f.startswith("seq_") and f.endswith(".npz"))
RTOL = 1e-8


@pytest.fixture(scope="module")
def fs():
    import torch  # noqa: F401  (loads the HIP runtime first)
    import fast_slam_2
    from gpu_util import configure
    yield fast_slam_2
    configure()


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def test_native_loaded(fs):
    from fast_slam_2 import _native
    lib = _native.load()
    assert lib.fs2_abi_version() == 2


def test_mahalanobis_bit_exact(fs):
    d = load("unit_geometry.npz")
    got = fs.GeometryUtils.mahalanobis_distances(d["a"], d["b"], d["cov"])
    assert np.array_equal(got, d["dist"])


def test_associate_golden(fs):
    d = load("unit_geometry.npz")
    from gpu_util import configure
    configure(gate=float(d["gate"]))
    for q in range(len(d["observed"])):
        lms = [fs.Landmark(d["lm"][q, j, 0], d["lm"][q, j, 1], d["lm_cov"][q, j])
               for j in range(d["lm"].shape[1])]
        lm, idx = fs.LandmarkUtils.associate_landmarks(
            fs.Landmark(d["observed"][q, 0], d["observed"][q, 1]), lms)
        exp = int(d["assoc"][q])
        assert (idx if idx is not None else -1) == exp, q
    configure()


def test_singular_raises(fs):
    with pytest.raises(np.linalg.LinAlgError):
        fs.GeometryUtils.mahalanobis_distance([0, 0], [1, 1], np.zeros((2, 2)))


def test_line_filter_golden(fs):
    d = load("unit_linefilter.npz")
    for k, s in enumerate(d["sigma"]):
        assert np.allclose(fs.LineFilter.filter(d["points"], s), d["out"][k], rtol=1e-14, atol=1e-14)
        assert np.allclose(fs.LineFilter.filter(d["short"], s), d["out_short"][k], rtol=1e-14,
                           atol=1e-14)
    assert np.array_equal(fs.LineFilter.filter(d["points"], 0.1), d["points"])


def test_best_fit_golden(fs):
    d = load("unit_bft.npz")
    for k in range(len(d["src"])):
        R, t = fs.ICP.best_fit_transform(d["src"][k], d["tgt"][k])
        assert np.allclose(R, d["R"][k], atol=1e-13)
        assert np.allclose(t, d["t"][k], atol=1e-12)


def _icp_cases():
    d = load("unit_icp.npz")
    k180 = k720 = 0
    for k, P in enumerate(d["P"]):
        if P == 180:
            yield k, d["src180"][k180], d["tgt180"][k180], d
            k180 += 1
        else:
            yield k, d["src720"][k720], d["tgt720"][k720], d
            k720 += 1


def test_icp_golden(fs):
    for k, src, tgt, d in _icp_cases():
        R, t, it = fs.ICP.get_transformation_ex(src, tgt)
        assert it == d["iters"][k], (k, it)
        assert np.allclose(R, d["R"][k], atol=1e-10)
        assert np.allclose(t, d["t"][k], atol=1e-10)


def test_icp_batched_matches_single(fs):
    cases = [c for c in _icp_cases() if len(c[1]) == 720]
    src = np.stack([c[1] for c in cases])
    tgt = np.stack([c[2] for c in cases])
    R, t, it = fs.ICP.get_transformation_batched(src, tgt)
    for b, (k, s, g, d) in enumerate(cases):
        assert it[b] == d["iters"][k]
        assert np.allclose(R[b], d["R"][k], atol=1e-10)
        assert np.allclose(t[b], d["t"][k], atol=1e-10)


def test_icp_submit_wait(fs):
    """The pipelined form (fs2_icp_submit / fs2_icp_wait) returns the golden
    alignments, out of order too; a fifth outstanding ticket and a ticket that
    is not outstanding are refused."""
    cases = list(_icp_cases())
    for lo in range(0, len(cases), 4):
        group = cases[lo:lo + 4]
        tickets = [fs.ICP.submit(src, tgt) for _, src, tgt, _ in group]
        # the caller's arrays may change once submit returns
        for _, src, tgt, _ in group:
            src[:] = np.nan
            tgt[:] = np.nan
        if len(group) == 4:
            with pytest.raises(RuntimeError):
                fs.ICP.submit(np.zeros((8, 2)), np.zeros((8, 2)))
        for (k, _, _, d), tk in reversed(list(zip(group, tickets))):
            R, t, it = tk.result()
            assert it == d["iters"][k], (k, it)
            assert np.allclose(R, d["R"][k], atol=1e-10)
            assert np.allclose(t, d["t"][k], atol=1e-10)
    from fast_slam_2 import _native as nat
    R, t = np.empty(4), np.empty(2)
    assert nat.load().fs2_icp_wait(0, tickets[0].ticket, nat.dptr(R), nat.dptr(t), None) == nat.FS2_ERR_STATE


@pytest.mark.parametrize("name", SEQS)
def test_sequence_golden(fs, name):
    from gpu_util import close, from_fixture
    d = load(f"seq_{name}.npz")
    f = from_fixture(d)
    S, cap = int(d["S"]), int(d["cap"])
    for s in range(S):
        M = int(d["M"][s])
        u0 = d["uniform"][s]
        pose, st = f.step(d["rotation"][s], d["translation"][s], d["meas"][s, :M],
                          d["observed"][s, :M], d["normals"][s],
                          0.0 if np.isnan(u0) else u0)
        assert st.error_flags == 0
        assert np.array_equal(f.associations(), d["assoc"][s, :M]), (name, s)
        assert bool(st.resampled) == (not np.isnan(u0)), (name, s)
        assert np.isclose(st.n_eff, d["n_eff"][s], rtol=1e-9), (name, s)
        assert close(pose, d["estimate"][s], RTOL), (name, s, pose, d["estimate"][s])
        x, y, yaw, w, cnt, lm = f.get_state(lm_cap=cap)
        assert np.array_equal(cnt, d["cnt"][s + 1]), (name, s)
        assert close(x, d["x"][s + 1], RTOL) and close(y, d["y"][s + 1], RTOL), (name, s)
        assert close(yaw, d["yaw"][s + 1], RTOL), (name, s)
        assert close(w, d["w"][s + 1], 1e-7, 0.0), (name, s)
        assert close(lm, d["lm"][s + 1], RTOL), (name, s)
    f.close()


def test_sequence_parallel_reduce(fs):
    """Same fixture through the parallel (tree) reductions: decisions unchanged."""
    from gpu_util import close, from_fixture
    d = load("seq_cfg1_n100_l20.npz")
    f = from_fixture(d, reduce="parallel")
    for s in range(int(d["S"])):
        M = int(d["M"][s])
        u0 = d["uniform"][s]
        pose, st = f.step(d["rotation"][s], d["translation"][s], d["meas"][s, :M],
                          d["observed"][s, :M], d["normals"][s], 0.0 if np.isnan(u0) else u0)
        assert np.array_equal(f.associations(), d["assoc"][s, :M])
        assert bool(st.resampled) == (not np.isnan(u0))
        assert close(pose, d["estimate"][s], RTOL)
    f.close()


def test_capacity_growth_and_state_roundtrip(fs):
    """Maps grow past the first 64-slot page; get/set state round-trips exactly."""
    from oracle import oracle as orc
    import fs2_synthetic as syn
    N, L = 300, 60
    wl = syn.Workload(N, L, seed=3)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    f = fs.FastSLAM2(N, reduce="sequential", record_assoc=True, landmark_capacity=8,
                     verbose=False)
    f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    x2, y2, yaw2, w2, c2, lm2 = f.get_state(lm_cap=L)
    assert np.array_equal(lm2, lm) and np.array_equal(x2, x) and np.array_equal(c2, np.full(N, L))
    o = orc.OracleFilter(N, 128)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    rng = np.random.default_rng(9)
    for s in range(8):     # 8 misses each scan -> 60 + 64 slots: crosses a page boundary
        ms = np.concatenate([syn.scan_measurements(L, s, 3, n_hits=3, with_miss=False),
                             np.array([syn.encode(*(syn.miss_point(L, 11 * s + q)))
                                       for q in range(8)])])
        rot, tr = syn.odometry(s)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        pose, st = f.step(rot, tr, ms, None, nz, 0.5 / N)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, 0.5 / N)
        assert np.array_equal(f.associations(), oassoc), s
        assert bool(st.resampled) == ors
        assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12)
    xg, yg, yawg, wg, cg, lmg = f.get_state(lm_cap=128)
    assert np.array_equal(cg, o.cnt)
    assert np.allclose(lmg, o.lm, rtol=RTOL, atol=1e-12)
    assert np.allclose(wg, o.w, rtol=1e-7, atol=0)
    f.close()


def test_zero_measurements_and_rotation(fs):
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L = 1000, 10
    wl = syn.Workload(N, L, seed=4)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    f = fs.FastSLAM2(N, reduce="sequential", record_assoc=True, verbose=False)
    f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, 32)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    rng = np.random.default_rng(1)
    for s, (rot, tr, M) in enumerate([(0.05, 0.0, 0), (-0.2, 0.0, 2), (0.0, 0.0, 0),
                                      (0.0, 0.03, 5), (3.0, 0.0, 1)]):
        ms = syn.scan_measurements(L, s, 4, n_hits=M)[:M]
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        pose, st = f.step(rot, tr, ms, None, nz, 0.3 / N)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, 0.3 / N)
        if M:
            assert np.array_equal(f.associations(), oassoc)
        assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12), s
    f.close()


def test_resample_never_hangs(fs):
    """Weights summing below u_{N-1} with w[N-1] = 0: the reference loops forever
    (SURVEY Q10); the device returns N-1 for the remaining slots."""
    N = 4
    f = fs.FastSLAM2(N, reduce="sequential", verbose=False)
    # 1e-6 stays un-divided (Q6), so the normalised weights sum to 0.99999975 and
    # u_3 = 0.2499999 + 0.75 exceeds every reachable prefix; N_eff = 1.88 < 2.
    w0 = np.array([0.5, 0.3, 1e-6, 0.0])
    f.set_state(np.arange(N, dtype=float), np.zeros(N), np.zeros(N), w0)
    pose, st = f.step(0.0, 0.0, np.zeros((0, 2)), None, np.zeros(N), 0.2499999)
    assert st.resampled == 1
    x, *_ = f.get_state()
    from oracle import oracle as orc
    src = orc.resample_src(orc.normalize(w0), 0.2499999)
    assert src.tolist() == [0, 0, 1, 3]
    assert np.array_equal(x.astype(int), src)
    f.close()


def test_gate_filter_is_exact(fs):
    """The fp32 gate mirror only skips slots that cannot match: with and without it
    every association, weight and landmark is bit-identical, and it skips most
    fp64 slot reads."""
    import fs2_synthetic as syn
    N, L = 4096, 80
    wl = syn.Workload(N, L, seed=11)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    rng = np.random.default_rng(4)
    # anisotropic and near-singular covariances exercise the conditioning guard
    th = rng.uniform(0, np.pi, (N, L))
    l1 = 10 ** rng.uniform(-4, -1, (N, L))
    l2 = l1 * 10 ** rng.uniform(0, 9, (N, L))
    c, s = np.cos(th), np.sin(th)
    lm[:, :, 2] = c * c * l1 + s * s * l2
    lm[:, :, 3] = c * s * (l1 - l2)
    lm[:, :, 4] = lm[:, :, 3] + rng.normal(0, 1e-18, (N, L))
    lm[:, :, 5] = s * s * l1 + c * c * l2
    fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False)
          for g in (True, False)]
    for f in fl:
        f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    for sc in range(6):
        rot, tr = syn.odometry(sc)
        ms = np.concatenate([wl.measurements(sc), rng.normal(0, 12, (3, 2))])
        ms[:, 0] = np.abs(ms[:, 0])
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        out = [f.step(rot, tr, ms, None, nz, 0.3 / N) for f in fl]
        a0, a1 = fl[0].associations(), fl[1].associations()
        assert np.array_equal(a0, a1), sc
        assert np.array_equal(out[0][0], out[1][0])
        assert out[0][1].candidates < out[1][1].candidates
    s0, s1 = fl[0].get_state(lm_cap=L + 64), fl[1].get_state(lm_cap=L + 64)
    for a, b in zip(s0, s1):
        assert np.array_equal(a, b, equal_nan=True)
    for f in fl:
        f.close()


def test_oracle_parity_n20000(fs):
    """N = 20000, L = 50, parallel reductions, 6 scans with injected draws."""
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L = 20000, 50
    wl = syn.Workload(N, L, seed=5)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    f = fs.FastSLAM2(N, reduce="parallel", record_assoc=True, verbose=False)
    f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, 64)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    rng = np.random.default_rng(2)
    for s in range(6):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = rng.uniform(0, 1.0 / N)
        cur = o.cnt.astype(np.int64)
        pose, st = f.step(rot, tr, ms, None, nz, u0)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        assert np.array_equal(f.associations(), oassoc), s
        # the reference's first-match scan: j + 1 landmarks for a match at j, the
        # whole map as it stood for an append
        ref = 0
        for k in range(len(ms)):
            hit = oassoc[k] >= 0
            ref += int(np.where(hit, oassoc[k] + 1, cur).sum())
            cur = cur + (~hit)
        assert st.reference_visits == ref, s
        assert 0 < st.pages_opened <= st.slots_visited
        assert bool(st.resampled) == ors, s
        assert np.isclose(st.n_eff, one, rtol=1e-9)
        assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12), s
    xg, yg, yawg, wg, cg, lmg = f.get_state(lm_cap=64)
    assert np.array_equal(cg, o.cnt)
    assert np.allclose(lmg, o.lm, rtol=RTOL, atol=1e-12)
    f.close()


def test_config2_n100k_l200(fs):
    """BASELINE config 2 size (N = 1e5, L = 200): two scans vs the oracle, exact
    associations, device Philox noise path exercised for a third scan."""
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L = 100_000, 200
    wl = syn.Workload(N, L, seed=6)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    f = fs.FastSLAM2(N, reduce="parallel", record_assoc=True, landmark_capacity=L + 8,
                     verbose=False)
    f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, L + 8)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    del lm
    rng = np.random.default_rng(3)
    for s in range(2):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        nz = rng.normal(0, 0.0055, N)
        pose, st = f.step(rot, tr, ms, None, nz, 0.5 / N)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, 0.5 / N)
        assert np.array_equal(f.associations(), oassoc), s
        assert bool(st.resampled) == ors
        assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12)
        assert st.ambiguous == 0
    xg, yg, yawg, wg, cg, lmg = f.get_state(lm_cap=L + 8)
    assert np.array_equal(cg, o.cnt)
    assert np.allclose(lmg, o.lm, rtol=RTOL, atol=1e-12)
    # device RNG path: deterministic per seed, one append per particle (the miss)
    pose1, st1 = f.step(0.0, 0.03, wl.measurements(2))
    assert st1.appends + st1.hits == 4 * N and st1.appends >= N
    f.close()


def test_config2_exact_mode_sequence(fs):
    """BASELINE config 2 (N = 1e5, L = 200) in the reduction mode bench.py runs it
    (reduce="auto": the reference's summation orders bit for bit above 4096
    particles), 8 scans with injected draws against the oracle: associations,
    resample decisions, N_eff, estimates, weights and maps every scan; at least
    one resample (fast_slam_2.py:161-199,212-223)."""
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L, S = 100_000, 200, 8
    wl = syn.Workload(N, L, seed=6)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    cap = L + 4 * S + 8
    f = fs.FastSLAM2(N, reduce="auto", record_assoc=True, landmark_capacity=cap, verbose=False)
    f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, cap)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    del lm
    rng = np.random.default_rng(31)
    resamples = 0
    for s in range(S):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = rng.uniform(0, 1.0 / N)
        pose, st = f.step(rot, tr, ms, None, nz, u0)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        assert np.array_equal(f.associations(), oassoc), s
        assert bool(st.resampled) == ors, s
        assert np.isclose(st.n_eff, one, rtol=1e-12), s     # device exp/log within an ulp of libm
        assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12), s
        assert st.ambiguous == 0 and st.reduce_ambiguous == 0, s
        resamples += st.resampled
        _, _, _, wg, cg, _ = f.get_state(lm_cap=0)
        assert np.array_equal(cg, o.cnt), s
        assert np.allclose(wg, o.w, rtol=RTOL, atol=0), s
    assert resamples >= 1
    xg, yg, yawg, wg, cg, lmg = f.get_state(lm_cap=cap)
    assert np.allclose(xg, o.x, rtol=RTOL, atol=1e-12) and np.allclose(yawg, o.yaw, rtol=RTOL, atol=1e-12)
    assert np.allclose(lmg, o.lm, rtol=RTOL, atol=1e-12)
    f.close()


def test_candidate_list_overflow(fs):
    """More than kMaxCand (16) candidate slots per particle: 40 landmarks crowd the
    first measurement's point while a far measurement matches nothing, so the
    exact kernel walks the whole truncated list and then resumes with an exact
    scan after its last entry.  Bit-identical with and without the gate filter,
    and equal to the oracle."""
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L = 2048, 100
    wl = syn.Workload(N, L, seed=17)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    rng = np.random.default_rng(8)
    ms = np.concatenate([wl.measurements(0)[:3], [[40.0, 2.0]]])
    ox, oy = ms[0, 0] * np.cos(ms[0, 1]), ms[0, 0] * np.sin(ms[0, 1])
    crowd = np.sort(rng.choice(L, 40, replace=False))
    lm[:, crowd, 0] = ox + rng.normal(0, 0.05, (N, 40))
    lm[:, crowd, 1] = oy + rng.normal(0, 0.05, (N, 40))
    lm[:, crowd, 2] = lm[:, crowd, 5] = 0.5
    lm[:, crowd, 3] = lm[:, crowd, 4] = 0.0
    fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False,
                       landmark_capacity=L + 16) for g in (True, False)]
    for f in fl:
        f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, L + 16)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    for sc in range(3):
        rot, tr = syn.odometry(sc)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = 0.4 / N
        out = [f.step(rot, tr, ms, None, nz, u0) for f in fl]
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        assert np.array_equal(fl[0].associations(), fl[1].associations()), sc
        assert np.array_equal(fl[0].associations(), oassoc), sc
        assert np.array_equal(out[0][0], out[1][0])
        assert np.allclose(out[0][0], opose, rtol=RTOL, atol=1e-12), sc
        assert out[0][1].candidates < out[1][1].candidates
    s0, s1 = fl[0].get_state(lm_cap=L + 16), fl[1].get_state(lm_cap=L + 16)
    for a, b in zip(s0, s1):
        assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(s0[4], o.cnt)
    assert np.allclose(s0[5], o.lm, rtol=RTOL, atol=1e-12)
    for f in fl:
        f.close()


def test_page_sharing_long_run(fs):
    """40 scans with frequent resampling: maps share pages after every resample and
    copy them on first write; the pool is collected and grown along the way.
    Every scan equals the oracle (which deep-copies maps like the reference)."""
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L = 3000, 30
    wl = syn.Workload(N, L, seed=23)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    lm[:, :, 2] = lm[:, :, 5] = 0.01           # peaked likelihoods: resample often
    cap = L + 4 * 40 + 8
    f = fs.FastSLAM2(N, reduce="parallel", record_assoc=True, verbose=False, landmark_capacity=8)
    f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, cap)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    rng = np.random.default_rng(12)
    resamples = cow = 0
    for s in range(40):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = rng.uniform(0, 1.0 / N)
        pose, st = f.step(rot, tr, ms, None, nz, u0)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        assert np.array_equal(f.associations(), oassoc), s
        assert bool(st.resampled) == ors, s
        assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12), s
        resamples += st.resampled
        cow += st.cow_pages
    assert resamples >= 5 and cow > 0
    assert st.collections >= 2
    xg, yg, yawg, wg, cg, lmg = f.get_state(lm_cap=cap)
    assert np.array_equal(cg, o.cnt)
    assert np.allclose(lmg, o.lm, rtol=RTOL, atol=1e-12)
    assert np.allclose(wg, o.w, rtol=RTOL, atol=1e-300)
    f.close()


def test_page_summary_extreme_coordinates(fs):
    """Page summaries store boxes on a power-of-two grid fitted to the imported
    maps, rounded outward: maps at |x| ~ 1e5, 6.5e4 and at tiny scales (1e-6, below
    the finest grid cell) must give the same associations and state with and
    without the filter."""
    N, L = 1024, 40
    rng = np.random.default_rng(31)
    for scale in (1e5, 6.55e4, 1e-6):
        lm = np.zeros((N, L, 6))
        base = rng.uniform(-1, 1, (L, 2)) * scale
        lm[:, :, 0:2] = base + rng.normal(0, 0.02 * scale, (N, L, 2))
        lm[:, :, 2] = lm[:, :, 5] = (0.1 * scale) ** 2
        ms = np.array([[np.hypot(*base[k]) * 1.001, np.arctan2(base[k, 1], base[k, 0])]
                       for k in (3, 17, 29)] + [[scale * 3.0, 0.5]])
        x = rng.normal(0, 0.01 * scale, N)
        y = rng.normal(0, 0.01 * scale, N)
        yaw = rng.normal(0, 0.01, N)
        fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False)
              for g in (True, False)]
        for f in fl:
            f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
        for sc in range(3):
            nz = rng.normal(0, 0.0055, N)
            out = [f.step(0.0, 0.03, ms, None, nz, 0.3 / N) for f in fl]
            assert np.array_equal(fl[0].associations(), fl[1].associations()), (scale, sc)
            assert np.array_equal(out[0][0], out[1][0])
        s0, s1 = fl[0].get_state(lm_cap=L + 16), fl[1].get_state(lm_cap=L + 16)
        for a, b in zip(s0, s1):
            assert np.array_equal(a, b, equal_nan=True)
        for f in fl:
            f.close()


def test_summary_grid_growth_and_saturation(fs):
    """The summary grid is fitted to the first import (a 10 m map: 1/8 m cells),
    grows when a later import reaches 600 m (every descriptor re-encoded), and
    landmarks appended 5 km away saturate the grid (unbounded boxes).  With and
    without the filter, and against the oracle: identical associations and state."""
    from oracle import oracle as orc
    N, L = 512, 24
    rng = np.random.default_rng(57)
    lm = np.zeros((N, L, 6))
    base = rng.uniform(-5, 5, (L, 2))
    lm[:, :, 0:2] = base + rng.normal(0, 0.02, (N, L, 2))
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    x, y, yaw = (rng.normal(0, s_, N) for s_ in (0.02, 0.02, 0.01))
    far = lm[N // 2:].copy()
    far[:, :, 0:2] *= 120.0                     # second import: extent ~600 m
    cap = L + 40
    fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False,
                       landmark_capacity=cap) for g in (True, False)]
    o = orc.OracleFilter(N, cap)
    full = np.concatenate([lm[:N // 2], far])
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), full)
    for f in fl:
        f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
        f.set_state(cnt=np.full(N - N // 2, L, np.int32), lm=far, first=N // 2)
    for sc in range(4):
        ks = rng.choice(L, 2, replace=False)
        ms = np.array([[np.hypot(*base[k]) * 1.01, np.arctan2(base[k, 1], base[k, 0])] for k in ks] +
                      [[5000.0 + 10.0 * sc, 0.3 * sc], [5000.0 + 10.0 * sc, 0.3 * sc + 0.001]])
        nz = rng.normal(0, 0.0055, N)
        u0 = 0.37 / N
        out = [f.step(0.0, 0.03, ms, None, nz, u0) for f in fl]
        opose, oassoc, _, _ = o.iterate(0.0, 0.03, ms, nz, u0)
        assert np.array_equal(fl[0].associations(), fl[1].associations()), sc
        assert np.array_equal(fl[0].associations(), oassoc), sc
        assert np.array_equal(out[0][0], out[1][0]), sc
        assert np.allclose(out[0][0], opose, rtol=1e-9, atol=1e-12), sc
    s0, s1 = fl[0].get_state(lm_cap=cap), fl[1].get_state(lm_cap=cap)
    for a, b in zip(s0, s1):
        assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(s0[4], o.cnt)
    assert np.allclose(s0[5], o.lm, rtol=1e-9, atol=1e-12)
    for f in fl:
        f.close()


def test_icp_grid_search_matches_brute_force(fs):
    """The grid nearest-neighbour search is exact: clustered clouds, duplicated
    target points (exact ties -> lowest index), sources far outside the target
    box and a degenerate (collinear) target cloud give the oracle's brute-force
    ICP result."""
    from oracle import oracle as orc
    rng = np.random.default_rng(77)
    cases = []
    tgt = rng.normal(0, 1, (600, 2)) * [8, 3]
    tgt[::7] = tgt[3]                                   # exact duplicates
    src = tgt[rng.permutation(600)[:500]] + rng.normal(0, 0.05, (500, 2))
    cases.append((src, tgt))
    cl = np.concatenate([rng.normal(c, 0.2, (120, 2)) for c in ([0, 0], [10, 2], [-5, 7])])
    cases.append((cl[::-1] * 1.01 + [0.3, -0.2], cl))
    far = rng.normal(0, 1, (256, 2))
    for sh in ([9.0, 0.0], [0.0, 12.0], [20.0, 20.0]):  # sources outside the target box
        cases.append((far + sh, far))
    line = np.stack([np.linspace(-5, 5, 300), np.zeros(300)], 1)
    cases.append((line + [0.01, 0.2], line))            # zero-height box
    for k, (s, t) in enumerate(cases):
        R, tt, it = fs.ICP.get_transformation_ex(s, t)
        Ro, to, ito = orc.icp(s, t)
        assert it == ito, k
        assert np.allclose(R, Ro, atol=1e-9), k
        assert np.allclose(tt, to, atol=1e-9 * max(1.0, np.abs(to).max())), k


def test_gate_band_boundaries(fs):
    """The measurement bands of the candidate stream (integer page pre-test on the
    summary codes, one-compare slot pre-test) only drop what the slot test drops:
    pages of landmarks just inside / just outside the gate radius along +-x, +-y
    and the diagonals, at three scales, give the same associations and state with
    and without the filter, and the oracle's."""
    from oracle import oracle as orc
    N = 1024
    rng = np.random.default_rng(91)
    eps = (-1e-7, 1e-7, 3e-6, 3e-5, 1e-4, 1e-3, 1e-2, 0.3)      # 8 per page
    dirs = [(1, 0), (-1, 0), (0, 1), (0, -1), (0.6, 0.8), (-0.8, 0.6)]
    for scale in (1.0, 40.0, 1e-3):
        sig = 0.1 * scale
        r = 8.0 * sig                                   # MAXIMUM_LANDMARK_DISTANCE 8, cov sig^2 I
        obs = np.array([[3.1, 2.2], [-1.7, 4.4], [0.35, -2.9]]) * scale
        base = np.array([o + np.array(d) * r * (1.0 + e) for o in obs for d in dirs for e in eps])
        L = len(base)                                    # 144 landmarks, 18 pages
        lm = np.zeros((N, L, 6))
        lm[:, :, 0:2] = base + rng.normal(0, sig * 1e-9, (N, L, 2))
        lm[:, :, 2] = lm[:, :, 5] = sig * sig
        x, y, yaw = (rng.normal(0, s_ * scale, N) for s_ in (1e-3, 1e-3, 1e-3))
        cap = L + 16
        fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False,
                           landmark_capacity=cap) for g in (True, False)]
        for f in fl:
            f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
        o = orc.OracleFilter(N, cap)
        o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
        for sc in range(3):
            ob = obs[[(sc + k) % 3 for k in range(3)]] + rng.normal(0, sig * 1e-9, (3, 2))
            ob = np.concatenate([ob, [[9.0 * scale, -9.0 * scale]]])
            ms = np.stack([np.hypot(ob[:, 0], ob[:, 1]), np.arctan2(ob[:, 1], ob[:, 0])], 1)
            nz = rng.normal(0, 0.0055 * scale, N)
            u0 = 0.41 / N
            out = [f.step(0.0, 0.03 * scale, ms, ob, nz, u0) for f in fl]
            opose, oassoc, _, _ = o.iterate(0.0, 0.03 * scale, ms, nz, u0, observed=ob)
            assert np.array_equal(fl[0].associations(), fl[1].associations()), (scale, sc)
            assert np.array_equal(fl[0].associations(), oassoc), (scale, sc)
            assert np.array_equal(out[0][0], out[1][0]), (scale, sc)
            assert out[0][1].candidates < out[1][1].candidates
        s0, s1 = fl[0].get_state(lm_cap=cap), fl[1].get_state(lm_cap=cap)
        for a, b in zip(s0, s1):
            assert np.array_equal(a, b, equal_nan=True)
        assert np.array_equal(s0[4], o.cnt)
        for f in fl:
            f.close()


def test_linalg_error_then_recover(fs):
    """A singular landmark covariance raises numpy.linalg.LinAlgError, as the
    reference's np.linalg.inv does (geometry_utils.py:21); after set_state the
    next scans match the oracle, and their statistics start clean (the failed
    scan's counters do not leak into the published stats)."""
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L = 512, 12
    wl = syn.Workload(N, L, seed=8)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    bad = lm.copy()
    bad[:, 3, 2:6] = 0.0                         # landmark 3 singular in every map
    f = fs.FastSLAM2(N, reduce="parallel", record_assoc=True, verbose=False)
    f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), bad)
    rng = np.random.default_rng(3)
    with pytest.raises(np.linalg.LinAlgError):   # the miss measurement scans every slot
        f.step(0.0, 0.03, wl.measurements(0), None, rng.normal(0, 0.0055, N), 0.3 / N)
    f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, L + 8)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    for s in range(2):
        ms = wl.measurements(s + 1)
        nz = rng.normal(0, 0.0055, N)
        pose, st = f.step(0.0, 0.03, ms, None, nz, 0.3 / N)
        opose, oassoc, _, _ = o.iterate(0.0, 0.03, ms, nz, 0.3 / N)
        assert np.array_equal(f.associations(), oassoc), s
        assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12), s
        assert st.appends == int((oassoc == -1).sum()), s
        assert st.hits == int((oassoc >= 0).sum()), s
    f.close()


def test_sweep_scan_tiles(fs):
    """k_sweep_scan (pool collection's exclusive scan of per-block free counts)
    across its 8192-count tiles, through libfs2_hooks.so: equal to numpy."""
    import ctypes as C
    hooks = os.path.join(os.path.dirname(fs.__file__), "..", "lib", "libfs2_hooks.so")
    lib = C.CDLL(os.path.abspath(hooks))
    lib.fs2_debug_sweep_scan.argtypes = [C.c_int32, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
    rng = np.random.default_rng(11)
    for nb in (1, 7, 1023, 8192, 8193, 34_700, 100_003):
        cnt = rng.integers(0, 4097, nb).astype(np.int64)
        cnt[rng.random(nb) < 0.1] = 0
        out = cnt.copy()
        tot = C.c_int64(-1)
        assert lib.fs2_debug_sweep_scan(0, out.ctypes.data, nb, C.byref(tot)) == 0
        assert tot.value == int(cnt.sum()), nb
        assert np.array_equal(out, np.concatenate([[0], np.cumsum(cnt)[:-1]])), nb


def _meas_at(pts):
    """Robot-frame (distance, angle) whose observed point is each (x, y): the
    association compares that point with world-frame landmarks."""
    pts = np.asarray(pts, float)
    return np.stack([np.hypot(pts[:, 0], pts[:, 1]), np.arctan2(pts[:, 1], pts[:, 0])], 1)


def test_row_boxes_follow_resampled_and_appended_maps(fs):
    """Workgroup row boxes (k_candidates skips rows whose workgroup box every band
    rejects): each of 8 workgroups' maps sits in its own region, so the boxes are
    tight and disjoint; peaked likelihoods then resample every output from the
    last workgroup's particles (the other workgroups' boxes must take its rows),
    and the misses append landmarks in new rows that later scans match.  Filter
    on / off bit-identical and equal to the oracle at every scan."""
    from oracle import oracle as orc
    N, L, cap = 2048, 24, 64
    rng = np.random.default_rng(41)
    centres = np.array([[30.0 * np.cos(a), 30.0 * np.sin(a)] for a in np.linspace(0, 2 * np.pi, 9)[:8]])
    lm = np.zeros((N, L, 6))
    for b in range(8):
        sl = slice(256 * b, 256 * b + 256)
        lm[sl, :, 0:2] = centres[b] + rng.uniform(-4, 4, (L, 2)) + rng.normal(0, 0.05, (256, L, 2))
    lm[:, :, 2] = lm[:, :, 5] = 0.02
    x = rng.normal(0, 0.05, N)
    y = rng.normal(0, 0.05, N)
    yaw = rng.normal(0, 0.01, N)
    fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False,
                       landmark_capacity=cap) for g in (True, False)]
    for f in fl:
        f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, cap)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    target = lm[N - 1, 5, 0:2]               # a landmark of the last workgroup's maps
    scans = [
        _meas_at([target, centres[0] + [60.0, 0.0]]),         # resample onto workgroup 7; one append
        _meas_at([target + [0.1, 0.1], centres[0]]),            # every particle now a copy of 7
        _meas_at([centres[0] + [60.0, 0.0], centres[3] + [9.0, 9.0]]),   # the appended landmark; a new one
        _meas_at([centres[3] + [9.0, 9.0], target]),
    ]
    resampled = hit = app = 0
    for sc, ms in enumerate(scans):
        rot, tr = (0.0, 0.02)
        nz = rng.normal(0, 0.0055, N)
        u0 = 0.37 / N
        out = [f.step(rot, tr, ms, None, nz, u0) for f in fl]
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        assert np.array_equal(fl[0].associations(), fl[1].associations()), sc
        assert np.array_equal(fl[0].associations(), oassoc), sc
        assert bool(out[0][1].resampled) == ors, sc
        assert np.allclose(out[0][0], opose, rtol=RTOL, atol=1e-12), sc
        resampled += out[0][1].resampled
        hit += int((oassoc >= 0).sum())
        app += int((oassoc == -1).sum())
    assert resampled >= 1 and hit > 0 and app > 0
    s0, s1 = fl[0].get_state(lm_cap=cap), fl[1].get_state(lm_cap=cap)
    for a, b in zip(s0, s1):
        assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(s0[4], o.cnt)
    assert np.allclose(s0[5], o.lm, rtol=RTOL, atol=1e-12)
    for f in fl:
        f.close()


def test_maps_beyond_row_boxes(fs):
    """Maps of more than 256 page rows (2048 slots) run without workgroup row
    boxes: filter on / off identical and equal to the oracle."""
    from oracle import oracle as orc
    N, L, cap = 300, 2100, 2112
    rng = np.random.default_rng(43)
    lm = np.zeros((N, L, 6))
    lm[:, :, 0:2] = rng.uniform(-50, 50, (L, 2)) + rng.normal(0, 0.05, (N, L, 2))
    lm[:, :, 2] = lm[:, :, 5] = 0.05
    x, y, yaw = (rng.normal(0, 0.05, N) for _ in range(3))
    fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False,
                       landmark_capacity=cap) for g in (True, False)]
    for f in fl:
        f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, cap)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    for sc in range(3):
        ms = _meas_at([lm[0, 2000 - 7 * sc, 0:2], lm[0, 17 + sc, 0:2], [80.0, 80.0]])
        nz = rng.normal(0, 0.0055, N)
        out = [f.step(0.0, 0.02, ms, None, nz, 0.5 / N) for f in fl]
        opose, oassoc, ors, one = o.iterate(0.0, 0.02, ms, nz, 0.5 / N)
        assert np.array_equal(fl[0].associations(), fl[1].associations()), sc
        assert np.array_equal(fl[0].associations(), oassoc), sc
        assert np.allclose(out[0][0], opose, rtol=RTOL, atol=1e-12), sc
    s0 = fl[0].get_state(lm_cap=cap)
    assert np.array_equal(s0[4], o.cnt)
    assert np.allclose(s0[5], o.lm, rtol=RTOL, atol=1e-12)
    for f in fl:
        f.close()


@pytest.mark.parametrize("order,wild", [((3, 0, 2, 1), False), ((0, 3, 1, 2), False), ((2, 0, 1, 3), True)])
def test_overflow_in_every_measurement_order(fs, order, wild):
    """Round 6: the overflow path in every measurement order.  Two crowds of 30
    (interleaved indices, tight to loose covariances) and a grid hit, with the far
    miss (no candidate: it is appended, then re-observed on the slot it appended)
    first, second or last; `wild`: an ill-conditioned slot (s = 0 mirror: a
    candidate of every measurement, never rejected) placed past the listed slots.
    Every scan equals the filter-off handle and the oracle (landmark_utils.py:92-117's
    first match with the map left by the earlier measurements)."""
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L, seed = 2048, 120, 5
    wl = syn.Workload(N, L, seed=seed)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    rng = np.random.default_rng(seed + 200)
    base = wl.measurements(0)
    ms4 = np.concatenate([base[:3], [[40.0, 2.0]]])
    idx = rng.permutation(L)[:60]
    for k, crowd in enumerate((idx[:30], idx[30:])):
        ox, oy = ms4[k, 0] * np.cos(ms4[k, 1]), ms4[k, 0] * np.sin(ms4[k, 1])
        lm[:, crowd, 0] = ox + rng.normal(0, 0.6, (N, 30))
        lm[:, crowd, 1] = oy + rng.normal(0, 0.6, (N, 30))
        v = np.exp(rng.uniform(np.log(0.005), np.log(0.5), (N, 30)))
        lm[:, crowd, 2] = lm[:, crowd, 5] = v
        lm[:, crowd, 3] = lm[:, crowd, 4] = 0.0
    if wild:
        j = L - 3                    # past every crowd's smallest slots
        lm[:, j, 2], lm[:, j, 5] = 1e-5, 1e4
        lm[:, j, 3] = lm[:, j, 4] = 0.0
    ms = ms4[list(order)]
    fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False,
                       landmark_capacity=L + 16) for g in (True, False)]
    for f in fl:
        f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, L + 16)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    for sc in range(4):
        rot, tr = syn.odometry(sc)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = 0.3 / N
        out = [f.step(rot, tr, ms, None, nz, u0) for f in fl]
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        assert np.array_equal(fl[0].associations(), oassoc), sc
        assert np.array_equal(fl[1].associations(), oassoc), sc
        assert np.array_equal(out[0][0], out[1][0]), sc
        assert np.allclose(out[0][0], opose, rtol=RTOL, atol=1e-12), sc
    s0, s1 = fl[0].get_state(lm_cap=L + 16), fl[1].get_state(lm_cap=L + 16)
    for a, b in zip(s0, s1):
        assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(s0[4], o.cnt)
    assert np.allclose(s0[5], o.lm, rtol=RTOL, atol=1e-12)
    for f in fl:
        f.close()


@pytest.mark.parametrize("seed", [3, 11])
def test_overflow_list_then_scan(fs, seed):
    """Round 5: an overflowing candidate list keeps its kMaxCand smallest slots, the
    exact kernel settles every measurement that matches among them in slot order and
    scans only past the last listed slot for the rest.  Two crowds of 30 landmarks
    (interleaved map indices, covariances from tight to loose so some crowd members
    pass the fp32 pre-test and fail the exact gate) around measurements 0 and 1, a
    grid hit, a far miss: the measurements' first matches fall before, among and
    after the listed slots; every scan equals the filter-off handle and the oracle
    (landmark_utils.py:92-117's first match with the map left by the earlier
    measurements)."""
    import fs2_synthetic as syn
    from oracle import oracle as orc
    N, L = 3000, 120
    wl = syn.Workload(N, L, seed=seed)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    rng = np.random.default_rng(seed + 100)
    base = wl.measurements(0)
    ms = np.concatenate([base[:3], [[40.0, 2.0]]])
    idx = rng.permutation(L)[:60]
    for k, crowd in enumerate((idx[:30], idx[30:])):
        ox, oy = ms[k, 0] * np.cos(ms[k, 1]), ms[k, 0] * np.sin(ms[k, 1])
        lm[:, crowd, 0] = ox + rng.normal(0, 0.6, (N, 30))
        lm[:, crowd, 1] = oy + rng.normal(0, 0.6, (N, 30))
        v = np.exp(rng.uniform(np.log(0.005), np.log(0.5), (N, 30)))
        lm[:, crowd, 2] = lm[:, crowd, 5] = v
        lm[:, crowd, 3] = lm[:, crowd, 4] = 0.0
    fl = [fs.FastSLAM2(N, reduce="parallel", record_assoc=True, gate_filter=g, verbose=False,
                       landmark_capacity=L + 16) for g in (True, False)]
    for f in fl:
        f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    o = orc.OracleFilter(N, L + 16)
    o.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L), lm)
    for sc in range(4):
        rot, tr = syn.odometry(sc)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = 0.3 / N
        out = [f.step(rot, tr, ms, None, nz, u0) for f in fl]
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        assert np.array_equal(fl[0].associations(), oassoc), sc
        assert np.array_equal(fl[1].associations(), oassoc), sc
        assert np.array_equal(out[0][0], out[1][0]), sc
        assert np.allclose(out[0][0], opose, rtol=RTOL, atol=1e-12), sc
    s0, s1 = fl[0].get_state(lm_cap=L + 16), fl[1].get_state(lm_cap=L + 16)
    for a, b in zip(s0, s1):
        assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(s0[4], o.cnt)
    assert np.allclose(s0[5], o.lm, rtol=RTOL, atol=1e-12)
    for f in fl:
        f.close()
