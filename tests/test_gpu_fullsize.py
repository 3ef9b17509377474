"""Parity at the BASELINE sizes: configs 3 and 4 (N = 1e6 particles, L = 500
landmarks, M = 4 measurements per scan) against the C oracle, scan by scan.

Config 3 (SURVEY §8d workload, 6 scans): injected motion normals and resample
starts; the pools are sized so that the page pool and the record pool are both
collected (and grown) inside the run, and the run resamples
(EXACT reductions: the reference's summation orders).  Every scan: the N x M
association indices and every map size bit-exact, the resample decision equal,
N_eff / pose / weights within 1e-9, sampled maps within 1e-9; at the end every
landmark of every particle within 1e-9.

Config 4 continues from that state with 720-beam scans: each scan's odometry is
the ICP alignment of the previous 720-point scan to this one, enqueued on the
ICP stream (Robot.submit_icp) and turned into (rotation, translation) by
Robot.icp_odometry (reference robot.py:93-120); the alignment is checked
against the oracle's ICP, and both filters take the same odometry.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, L, M = 1_000_000, 500, 4
S3, S4 = 6, 2
CAP = L + M * (S3 + S4) + 8
RTOL = 1e-9


def _chunks(n, k):
    for a in range(0, n, k):
        yield a, min(n, a + k)


@pytest.fixture(scope="module")
def pair():
    import torch
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    from gpu_util import configure
    from oracle import oracle as orc
    configure()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(31337)
    base = torch.tensor(syn.common_landmarks(L, 0), dtype=torch.float64, device=dev)
    x = torch.randn(N, generator=g, dtype=torch.float64, device=dev) * 0.05
    y = torch.randn(N, generator=g, dtype=torch.float64, device=dev) * 0.05
    yaw = torch.randn(N, generator=g, dtype=torch.float64, device=dev) * 0.01
    # weights of a filter some scans in (SURVEY §8d starts from 1/N): spread enough
    # that the N_eff < N/2 rule fires on some scans and not on others
    wh = np.random.default_rng(77).lognormal(0.0, 0.85, N)
    w = torch.tensor(wh / wh.sum(), dtype=torch.float64, device=dev)
    rows = (L + 7) // 8
    # pools just above the imported maps: both are collected (and grown) in the run
    f = fast_slam_2.FastSLAM2(N, record_assoc=True, landmark_capacity=CAP, verbose=False,
                              page_pool=N * rows + 6 * N, record_pool=N * L + 10 * N)
    o = orc.OracleFilter(N, CAP)
    torch.cuda.synchronize()
    nat.check(f._lib.fs2_set_state(f._h, 0, N, x.data_ptr(), y.data_ptr(), yaw.data_ptr(), w.data_ptr(),
                                   None, None, 0, nat.FS2_DEVICE), f._h)
    o.x[:], o.y[:], o.yaw[:], o.w[:] = (t.cpu().numpy() for t in (x, y, yaw, w))
    o.cnt[:] = L
    for a, b in _chunks(N, 100_000):
        k = b - a
        lm = torch.empty((k, L, 6), dtype=torch.float64, device=dev)
        lm[:, :, 0:2] = base + syn.MAP_JITTER * torch.randn((k, L, 2), generator=g, dtype=torch.float64,
                                                            device=dev)
        lm[:, :, 2] = lm[:, :, 5] = syn.INIT_COV
        lm[:, :, 3] = lm[:, :, 4] = 0.0
        cnt = torch.full((k,), L, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        nat.check(f._lib.fs2_set_state(f._h, a, k, None, None, None, None, cnt.data_ptr(), lm.data_ptr(), L,
                                       nat.FS2_DEVICE), f._h)
        o.lm[a:b, :L] = lm.cpu().numpy()
        del lm, cnt
    torch.cuda.synchronize()
    state = dict(f=f, o=o, rng=np.random.default_rng(8), resamples=0, scan=0)
    yield state
    f.close()
    del state["o"]


def _check_scan(f, o, st, pose, opose, oassoc, ors, one, rng, tag):
    assert st.error_flags == 0, tag
    assert np.array_equal(f.associations(), oassoc), tag
    assert bool(st.resampled) == ors, tag
    assert np.isclose(st.n_eff, one, rtol=RTOL), tag
    assert np.allclose(pose, opose, rtol=RTOL, atol=1e-12), tag
    x, y, yaw, w, cnt, _ = f.get_state(lm_cap=0)
    assert np.array_equal(cnt, o.cnt), tag
    assert np.allclose(x, o.x, rtol=RTOL, atol=1e-12) and np.allclose(y, o.y, rtol=RTOL, atol=1e-12), tag
    assert np.allclose(yaw, o.yaw, rtol=RTOL, atol=1e-12), tag
    assert np.allclose(w, o.w, rtol=RTOL, atol=1e-300), tag
    # a few windows of whole maps every scan
    for a in (0, int(rng.integers(0, N - 2048)), N - 2048):
        lm = f.get_state(first=a, count=2048, lm_cap=CAP)[5]
        assert np.allclose(lm, o.lm[a:a + 2048], rtol=RTOL, atol=1e-12), (tag, a)


def _final_maps(f, o):
    for a, b in _chunks(N, 50_000):
        lm = f.get_state(first=a, count=b - a, lm_cap=CAP)[5]
        assert np.allclose(lm, o.lm[a:b], rtol=RTOL, atol=1e-12), a


@pytest.mark.timeout(400)
def test_config3_full_size(pair):
    import fs2_synthetic as syn
    f, o, rng = pair["f"], pair["o"], pair["rng"]
    for s in range(S3):
        rot, tr = syn.odometry(s)
        ms = syn.scan_measurements(L, s, 0)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = rng.uniform(0, 1.0 / N)
        pose, st = f.step(rot, tr, ms, None, nz, u0)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        _check_scan(f, o, st, pose, opose, oassoc, ors, one, rng, ("cfg3", s))
        assert st.reduce_ambiguous == 0
        pair["resamples"] += st.resampled
    pair["scan"] = S3
    assert pair["resamples"] >= 1
    assert st.collections >= 2          # page pool, then pages + records
    _final_maps(f, o)


@pytest.mark.timeout(300)
def test_config4_icp_full_size(pair):
    import fast_slam_2
    import fs2_synthetic as syn
    from oracle import oracle as orc
    f, o, rng = pair["f"], pair["o"], pair["rng"]
    assert pair["scan"] == S3, "runs after test_config3_full_size"
    pose_true = [0.0, 0.0, 0.0]
    pts = syn.room_scan(tuple(pose_true), 720, 0, 0)
    robot = fast_slam_2.Robot(prev_points=pts)
    for k in range(S4):
        s = S3 + k
        rot_cmd, tr_cmd = syn.odometry(s)
        pose_true[2] += rot_cmd
        pose_true[0] += tr_cmd * np.cos(pose_true[2])
        pose_true[1] += tr_cmd * np.sin(pose_true[2])
        prev = robot._prev_points
        cur = syn.room_scan(tuple(pose_true), 720, 0, s)
        R, t, it = robot.submit_icp(cur).result()
        Ro, to, ito = orc.icp(prev, cur)
        assert it == ito and np.allclose(R, Ro, atol=1e-9) and np.allclose(t, to, atol=1e-9), s
        v = 0.3 if tr_cmd != 0 else 0.0
        rot, tr = (float(q) for q in fast_slam_2.Robot.icp_odometry(R, t, v))
        ms = syn.scan_measurements(L, s, 0)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = rng.uniform(0, 1.0 / N)
        pose, st = f.step(rot, tr, ms, None, nz, u0)
        opose, oassoc, ors, one = o.iterate(rot, tr, ms, nz, u0)
        _check_scan(f, o, st, pose, opose, oassoc, ors, one, rng, ("cfg4", s))
    _final_maps(f, o)
