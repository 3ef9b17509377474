"""The drop-in Python API against the reference's own outputs.

  * FastSLAM2.iterate(rotation, translation, [Measurement]) with numpy's legacy
    global RNG, as jde_robots_main.py:38 calls it: seeded like the golden run,
    the N motion normals and the speculative resample start (drawn before the
    scan, rewound when no resample fires) must replay the reference's stream
    (fast_slam_2.py:79-81, :183), so every scan's estimate,
    associations, map sizes and final state equal the fixture.
  * Robot.get_transformation_icp (robot.py:93-120) on the reference's outputs
    (tests/golden/gen_robot.py).
  * FastSLAM2.particles: the setter and the lazy view round-trip the state.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

SEQS = sorted(f[4:-4] for f in os.listdir(GOLDEN) if f.startswith("seq_") and f.endswith(".npz"))


@pytest.fixture(scope="module")
def fs():
    import torch  # noqa: F401
    import fast_slam_2
    from gpu_util import configure
    yield fast_slam_2
    configure()


@pytest.mark.parametrize("rng", ["numpy", "numpy-host"])
@pytest.mark.parametrize("name", SEQS)
def test_iterate_numpy_rng_replays_reference(fs, name, rng):
    """rng="numpy" draws numpy's stream on the GPU (fs2_mt_draw), "numpy-host" with numpy."""
    from gpu_util import close, configure
    d = np.load(os.path.join(GOLDEN, f"seq_{name}.npz"))
    tr, rot, mn = d["noise_cfg"]
    configure(tr, rot, mn, float(d["gate"]))
    N, cap = int(d["N"]), int(d["cap"])
    f = fs.FastSLAM2(N, record_assoc=True, landmark_capacity=cap, verbose=False, rng=rng)
    f.set_state(d["x"][0], d["y"][0], d["yaw"][0], d["w"][0], d["cnt"][0], d["lm"][0])
    np.random.seed(int(d["seed"]))
    for s in range(int(d["S"])):
        M = int(d["M"][s])
        ms = [fs.Measurement(float(a), float(b)) for a, b in d["meas"][s, :M]]
        pose = f.iterate(float(d["rotation"][s]), float(d["translation"][s]), ms)
        st = f.last_stats
        assert bool(st.resampled) == (not np.isnan(d["uniform"][s])), (name, s)
        if M:
            assert np.array_equal(f.associations(), d["assoc"][s, :M]), (name, s)
        assert close(np.array(pose), d["estimate"][s], 1e-8), (name, s, pose)
        x, y, yaw, w, cnt, lm = f.get_state(lm_cap=cap)
        assert np.array_equal(cnt, d["cnt"][s + 1]), (name, s)
        assert close(x, d["x"][s + 1], 1e-8) and close(yaw, d["yaw"][s + 1], 1e-8), (name, s)
        assert close(lm, d["lm"][s + 1], 1e-8), (name, s)
    # the global stream is where the reference left it: the next draw matches a
    # replay of the recorded draws from the same seed
    nxt = np.random.random()
    np.random.seed(int(d["seed"]))
    for s in range(int(d["S"])):
        np.random.normal(0, 1.0, size=N)
        if not np.isnan(d["uniform"][s]):
            np.random.uniform(0, 1 / N)
    assert nxt == np.random.random()
    f.close()


def test_robot_icp_odometry_golden(fs):
    d = np.load(os.path.join(GOLDEN, "unit_robot_icp.npz"))
    for k in range(len(d["v"])):
        prev = d["prev"][k, :d["n_prev"][k]]
        tgt = d["target"][k, :d["n_target"][k]]
        robot = fs.Robot(prev_points=prev)
        rot, tr = robot.get_transformation_icp(tgt, float(d["v"][k]))
        assert abs(rot - d["rotation"][k]) <= 1e-10, (k, rot)
        assert abs(tr - d["translation"][k]) <= 1e-10, (k, tr)
        # the next alignment starts from this target (robot.py:106)
        assert np.array_equal(robot._prev_points, tgt)
        # pipelined form: same result through the device's ICP stream
        r2 = fs.Robot(prev_points=prev)
        R, t, _ = r2.submit_icp(tgt).result()
        rot2, tr2 = fs.Robot.icp_odometry(R, t, float(d["v"][k]))
        assert rot2 == rot and tr2 == tr


def test_particles_setter_and_view_roundtrip(fs):
    import fs2_synthetic as syn
    N, L = 20_000, 12
    wl = syn.Workload(N, L, seed=41)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    rng = np.random.default_rng(3)
    w = rng.random(N)
    cnt = rng.integers(0, L + 1, N).astype(np.int32)
    plist = []
    for i in range(N):
        p = fs.Particle.__new__(fs.Particle)
        p.x, p.y, p.yaw, p.weight = float(x[i]), float(y[i]), float(yaw[i]), float(w[i])
        p.landmarks = [fs.Landmark(float(lm[i, j, 0]), float(lm[i, j, 1]), lm[i, j, 2:6].reshape(2, 2).copy())
                       for j in range(int(cnt[i]))]
        plist.append(p)
    f = fs.FastSLAM2(N, verbose=False)
    f.particles = plist
    xs, ys, yaws, ws, cs, lms = f.get_state(lm_cap=L)
    assert np.array_equal(xs, x) and np.array_equal(ws, w) and np.array_equal(cs, cnt)
    mask = np.arange(L)[None, :] < cnt[:, None]
    assert np.array_equal(lms[mask], lm[mask])
    view = f.particles
    assert len(view) == N
    for i in (0, 1, 4095, 4096, N // 2, N - 1):
        p = view[i]
        assert (p.x, p.y, p.yaw, p.weight) == (x[i], y[i], yaw[i], w[i])
        assert len(p.landmarks) == cnt[i]
        for j, l in enumerate(p.landmarks):
            assert (l.x, l.y) == (lm[i, j, 0], lm[i, j, 1])
            assert np.array_equal(np.asarray(l.cov).reshape(4), lm[i, j, 2:6])
    f.close()
