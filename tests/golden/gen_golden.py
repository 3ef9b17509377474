#!/usr/bin/env python3
"""Generate golden fixtures by running the reference CPU path (this container only).

The reference (cy-rae/fast-slam, pure Python) is imported from /root/reference
with empty stub modules for `HAL` (simulator API) and `cv2` (unused on the hot
path) -- SURVEY.md §8(c).  Nothing from the reference is copied: only its
outputs on seeded synthetic inputs are written to tests/golden/*.npz.

Instrumentation (all non-perturbing):
  * config knobs patched by name in every importing module;
    NUM_THREAD = 1 so the pool runs particles in index order (Q16);
  * numpy.random.normal / uniform wrapped to record every draw (Q4, Q5);
  * LandmarkUtils.associate_landmarks wrapped to record the association index
    per (measurement, particle) (landmark_utils.py:92-117);
  * FastSLAM2.__calculate_effective_particles wrapped to record N_eff;
  * a SIGALRM watchdog because the reference resample can hang (Q10).

Run:  python tests/golden/gen_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import importlib.util
import os
import signal
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

spec = importlib.util.spec_from_file_location(
    "fs2_synthetic", os.path.join(REPO, "fast-slam_amd", "fs2_synthetic.py"))
syn = importlib.util.module_from_spec(spec)
sys.modules["fs2_synthetic"] = syn
spec.loader.exec_module(syn)


def import_reference():
    sys.modules.setdefault("HAL", types.ModuleType("HAL"))
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, REF)
    import fast_slam_2  # noqa: F401
    import fast_slam_2.algorithms.fast_slam_2 as fs_mod
    import fast_slam_2.models.particle as particle_mod
    import fast_slam_2.utils.landmark_utils as lu_mod
    return fast_slam_2, fs_mod, particle_mod, lu_mod


fast_slam_2, fs_mod, particle_mod, lu_mod = import_reference()
from fast_slam_2 import (FastSLAM2, ICP, Landmark, LandmarkUtils,  # noqa: E402
                         LineFilter, Measurement, GeometryUtils)

VERSIONS = dict(numpy=np.__version__)
try:
    import scipy
    VERSIONS["scipy"] = scipy.__version__
except Exception:  # pragma: no cover
    pass


class Recorder:
    def __init__(self):
        self.normals, self.uniforms, self.assoc, self.neff = [], [], [], []
        self._normal = np.random.normal
        self._uniform = np.random.uniform
        self._assoc = LandmarkUtils.associate_landmarks
        self._neff = FastSLAM2._FastSLAM2__calculate_effective_particles

    def install(self):
        rec = self

        def normal(*a, **k):
            v = rec._normal(*a, **k)
            rec.normals.append(float(v))
            return v

        def uniform(*a, **k):
            v = rec._uniform(*a, **k)
            rec.uniforms.append(float(v))
            return v

        def assoc(observed, lms):
            lm, idx = rec._assoc(observed, lms)
            rec.assoc.append(-1 if idx is None else int(idx))
            return lm, idx

        def neff(self_):
            v = rec._neff(self_)
            rec.neff.append(float(v))
            return v

        np.random.normal = normal
        np.random.uniform = uniform
        LandmarkUtils.associate_landmarks = staticmethod(assoc)
        FastSLAM2._FastSLAM2__calculate_effective_particles = neff

    def uninstall(self):
        np.random.normal = self._normal
        np.random.uniform = self._uniform
        LandmarkUtils.associate_landmarks = staticmethod(self._assoc)
        FastSLAM2._FastSLAM2__calculate_effective_particles = self._neff

    def reset(self):
        self.normals, self.uniforms, self.assoc, self.neff = [], [], [], []


def configure(N, gate=8, tr_noise=0.0055, rot_noise=0.001, meas_noise=1e-3):
    """Patch config knobs where they were bound by name."""
    fs_mod.NUM_PARTICLES = N
    fs_mod.NUM_THREAD = 1
    fs_mod.TRANSLATION_NOISE = tr_noise
    fs_mod.ROTATION_NOISE = rot_noise
    fs_mod.MEASUREMENT_NOISE = np.array([[meas_noise, 0.0], [0.0, meas_noise]])
    particle_mod.NUM_PARTICLES = N
    lu_mod.MAXIMUM_LANDMARK_DISTANCE = gate


class Hang(Exception):
    pass


def _alarm(signum, frame):
    raise Hang()


def snapshot(fs, cap):
    N = len(fs.particles)
    x = np.array([float(p.x) for p in fs.particles])
    y = np.array([float(p.y) for p in fs.particles])
    yaw = np.array([float(p.yaw) for p in fs.particles])
    w = np.array([float(p.weight) for p in fs.particles])
    cnt = np.array([len(p.landmarks) for p in fs.particles], dtype=np.int32)
    lm = np.zeros((N, cap, 6))
    for i, p in enumerate(fs.particles):
        for j, l in enumerate(p.landmarks):
            c = np.asarray(l.cov, dtype=np.float64)
            lm[i, j] = (float(l.x), float(l.y), c[0, 0], c[0, 1], c[1, 0], c[1, 1])
    return x, y, yaw, w, cnt, lm


def populate(fs, x, y, yaw, w, cnt, lm):
    for i, p in enumerate(fs.particles):
        p.x, p.y, p.yaw, p.weight = float(x[i]), float(y[i]), float(yaw[i]), float(w[i])
        p.landmarks = [Landmark(float(lm[i, j, 0]), float(lm[i, j, 1]),
                                np.array([[lm[i, j, 2], lm[i, j, 3]], [lm[i, j, 4], lm[i, j, 5]]]))
                       for j in range(int(cnt[i]))]


def observed_points(meas):
    """The reference's observed robot-frame point (fast_slam_2.py:100-103)."""
    out = np.zeros((len(meas), 2))
    for k, (d, b) in enumerate(meas):
        m = Measurement(float(d), float(b))
        out[k, 0] = m.distance * np.cos(m.yaw)
        out[k, 1] = m.distance * np.sin(m.yaw)
    return out


def run_sequence(name, N, init, scans, seed, cap, gate=8, noises=None, timeout=120):
    """Run `scans` = [(rotation, translation, meas Mx2)] through the reference."""
    configure(N, gate=gate, **(noises or {}))
    np.random.seed(seed)
    fs = FastSLAM2()
    if init is not None:
        populate(fs, *init)
    rec = Recorder()
    rec.install()
    S = len(scans)
    Mmax = max([len(s[2]) for s in scans] + [1])
    st = [snapshot(fs, cap)]
    normals = np.full((S, N), np.nan)
    uniforms = np.full(S, np.nan)
    assoc = np.full((S, Mmax, N), -2, dtype=np.int32)
    meas = np.full((S, Mmax, 2), np.nan)
    obs = np.full((S, Mmax, 2), np.nan)
    Ms = np.zeros(S, dtype=np.int32)
    rot = np.zeros(S)
    tr = np.zeros(S)
    est = np.zeros((S, 3))
    neff = np.full(S, np.nan)
    hang = -1
    signal.signal(signal.SIGALRM, _alarm)
    try:
        for s, (r, t, ms) in enumerate(scans):
            rec.reset()
            M = len(ms)
            Ms[s], rot[s], tr[s] = M, r, t
            meas[s, :M] = ms
            obs[s, :M] = observed_points(ms)
            signal.alarm(timeout)
            try:
                e = fs.iterate(r, t, [Measurement(float(d), float(b)) for d, b in ms])
            except Hang:
                hang = s
                print(f"[{name}] reference hung at scan {s} (Q10)")
                break
            finally:
                signal.alarm(0)
            assert len(rec.normals) == N, (len(rec.normals), N)
            normals[s] = rec.normals
            if rec.uniforms:
                uniforms[s] = rec.uniforms[0]
            assoc[s, :M] = np.array(rec.assoc, dtype=np.int32).reshape(M, N)
            neff[s] = rec.neff[0]
            est[s] = [float(v) for v in e]
            st.append(snapshot(fs, cap))
    finally:
        rec.uninstall()
    S_done = len(st) - 1
    out = dict(
        N=N, S=S_done, gate=gate, seed=seed, cap=cap, hang_scan=hang,
        M=Ms[:S_done], rotation=rot[:S_done], translation=tr[:S_done],
        meas=meas[:S_done], observed=obs[:S_done], normals=normals[:S_done],
        uniform=uniforms[:S_done], assoc=assoc[:S_done], estimate=est[:S_done],
        n_eff=neff[:S_done],
        x=np.stack([q[0] for q in st]), y=np.stack([q[1] for q in st]),
        yaw=np.stack([q[2] for q in st]), w=np.stack([q[3] for q in st]),
        cnt=np.stack([q[4] for q in st]), lm=np.stack([q[5] for q in st]),
        noise_cfg=np.array([(noises or {}).get("tr_noise", 0.0055),
                            (noises or {}).get("rot_noise", 0.001),
                            (noises or {}).get("meas_noise", 1e-3)]),
        versions=np.array(repr(VERSIONS)),
    )
    np.savez_compressed(os.path.join(HERE, f"seq_{name}.npz"), **out)
    nres = int(np.sum(~np.isnan(uniforms[:S_done])))
    print(f"[{name}] N={N} scans={S_done} resamples={nres} maxcnt={int(st[-1][4].max())}")
    return out


def grid_init(N, L, seed, cap, pose_offset=(0.0, 0.0)):
    wl = syn.Workload(N, L, seed)
    x, y, yaw = wl.poses()
    x = x + pose_offset[0]
    y = y + pose_offset[1]
    w = np.full(N, 1.0 / N)
    lm = np.zeros((N, cap, 6))
    lm[:, :L] = wl.maps()
    cnt = np.full(N, L, dtype=np.int32)
    return x, y, yaw, w, cnt, lm


def gen_sequences():
    # A) room corners from an empty map (reference initial state), N = 20.
    pose = [0.0, 0.0, 0.0]
    scans = []
    for s in range(30):
        r, t = syn.odometry(s)
        pose[2] = (pose[2] + r + np.pi) % (2 * np.pi) - np.pi
        pose[0] += t * np.cos(pose[2])
        pose[1] += t * np.sin(pose[2])
        ms = syn.corner_measurements(tuple(pose), s, seed=11) if s % 7 != 3 else np.zeros((0, 2))
        scans.append((r, t, ms))
    run_sequence("room_n20", 20, None, scans, seed=1234, cap=64)

    # B) BASELINE config 1: N=100, L=20 grid maps, M=4 (3 hits + 1 miss).
    N, L = 100, 20
    init = grid_init(N, L, 0, cap=40)
    scans = [(*syn.odometry(s), syn.scan_measurements(L, s, 0)) for s in range(12)]
    run_sequence("cfg1_n100_l20", N, init, scans, seed=7, cap=40)

    # C) resample stress: peaked likelihoods (small landmark covariances), rotations.
    N, L = 64, 12
    x, y, yaw, w, cnt, lm = grid_init(N, L, 3, cap=40)
    lm[:, :L, 2] = lm[:, :L, 5] = 0.02
    scans = []
    for s in range(16):
        r, t = (0.05, 0.0) if s % 3 == 2 else (0.0, 0.03)
        scans.append((r, t, syn.scan_measurements(L, s, 3, n_hits=3, with_miss=(s % 4 == 0))))
    run_sequence("resample_n64", N, (x, y, yaw, w, cnt, lm), scans, seed=99, cap=40,
                 noises=dict(meas_noise=1e-4))

    # D) total weight collapses below 1e-5 -> every weight reset to 1/N (Q6).
    N, L = 32, 9
    init = grid_init(N, L, 5, cap=24, pose_offset=(4.0, -3.0))
    scans = [(*syn.odometry(s), syn.scan_measurements(L, s, 5, n_hits=2, with_miss=False))
             for s in range(5)]
    run_sequence("collapse_n32", N, init, scans, seed=5, cap=24)

    # E) weights straddling the 1e-5 floor (undivided small weights, Q6/Q8).
    N, L = 48, 9
    x, y, yaw, w, cnt, lm = grid_init(N, L, 6, cap=24)
    rng = np.random.default_rng(66)
    x = x + rng.normal(0, 0.6, N)
    y = y + rng.normal(0, 0.6, N)
    scans = [(*syn.odometry(s), syn.scan_measurements(L, s, 6, n_hits=2, with_miss=True))
             for s in range(8)]
    run_sequence("floor_n48", N, (x, y, yaw, w, cnt, lm), scans, seed=66, cap=24)

    # F) gate != 8 and larger N: N=1000, L=30, 3 scans.
    N, L = 1000, 30
    init = grid_init(N, L, 8, cap=36)
    scans = [(*syn.odometry(s), syn.scan_measurements(L, s, 8)) for s in range(3)]
    run_sequence("medium_n1000", N, init, scans, seed=8, cap=36, gate=6)


def gen_units():
    rng = np.random.default_rng(2024)
    # Mahalanobis distance (geometry_utils.py:13-23).
    K = 400
    a = rng.normal(0, 5, (K, 2))
    b = a + rng.normal(0, 1.5, (K, 2))
    covs = np.empty((K, 2, 2))
    for k in range(K):
        A = rng.normal(0, 0.4, (2, 2))
        covs[k] = A @ A.T + 0.01 * np.eye(2)
        covs[k, 0, 1] += rng.normal(0, 1e-3)  # asymmetric like EKF output (Q12)
    d = np.array([GeometryUtils.mahalanobis_distance(a[k], b[k], covs[k]) for k in range(K)])
    # Association (landmark_utils.py:92-117): first match in list order.
    Q, L = 200, 16
    lms = rng.normal(0, 4, (Q, L, 2))
    lcov = np.empty((Q, L, 2, 2))
    for q in range(Q):
        for j in range(L):
            A = rng.normal(0, 0.5, (2, 2))
            lcov[q, j] = A @ A.T + 0.05 * np.eye(2)
    obs = lms[np.arange(Q), rng.integers(0, L, Q)] + rng.normal(0, 2.0, (Q, 2))
    idx = np.empty(Q, dtype=np.int32)
    for q in range(Q):
        lst = [Landmark(lms[q, j, 0], lms[q, j, 1], lcov[q, j]) for j in range(L)]
        _, i = LandmarkUtils.associate_landmarks(Landmark(obs[q, 0], obs[q, 1]), lst)
        idx[q] = -1 if i is None else i
    np.savez_compressed(os.path.join(HERE, "unit_geometry.npz"), a=a, b=b, cov=covs, dist=d,
                        lm=lms, lm_cov=lcov, observed=obs, assoc=idx, gate=8.0,
                        versions=np.array(repr(VERSIONS)))

    # ICP (icp.py:13-90) on synthetic room scans, 180 and 720 beams.
    cases = []
    for P in (180, 720):
        for c in range(4):
            prev = syn.room_scan((0.0, 0.0, 0.0), P, seed=40 + c, scan=0)
            mv = [(0.03, 0.0, 0.0), (0.0, 0.0, 0.05), (0.06, 0.02, -0.03), (0.0, 0.1, 0.0)][c]
            cur = syn.room_scan(mv, P, seed=40 + c, scan=1)
            n_bft = [0]
            orig = ICP.best_fit_transform

            def counting(s_, t_, _o=orig):
                n_bft[0] += 1
                return _o(s_, t_)
            ICP.best_fit_transform = staticmethod(counting)
            try:
                R, t = ICP.get_transformation(prev.copy(), cur.copy())
            finally:
                ICP.best_fit_transform = staticmethod(orig)
            cases.append((P, prev, cur, R, t, n_bft[0]))
    np.savez_compressed(
        os.path.join(HERE, "unit_icp.npz"),
        P=np.array([c[0] for c in cases]),
        src180=np.stack([c[1] for c in cases if c[0] == 180]),
        tgt180=np.stack([c[2] for c in cases if c[0] == 180]),
        src720=np.stack([c[1] for c in cases if c[0] == 720]),
        tgt720=np.stack([c[2] for c in cases if c[0] == 720]),
        R=np.stack([c[3] for c in cases]), t=np.stack([c[4] for c in cases]),
        iters=np.array([c[5] for c in cases]), versions=np.array(repr(VERSIONS)))
    # best_fit_transform on random correspondences.
    B = 50
    src = rng.normal(0, 3, (B, 30, 2))
    th = rng.uniform(-np.pi, np.pi, B)
    tgt = np.empty_like(src)
    Rs, ts = [], []
    for k in range(B):
        Rk = np.array([[np.cos(th[k]), -np.sin(th[k])], [np.sin(th[k]), np.cos(th[k])]])
        tgt[k] = src[k] @ Rk.T + rng.normal(0, 1, 2) + rng.normal(0, 0.05, (30, 2))
        R, t = ICP.best_fit_transform(src[k], tgt[k])
        Rs.append(R)
        ts.append(t)
    np.savez_compressed(os.path.join(HERE, "unit_bft.npz"), src=src, tgt=tgt,
                        R=np.stack(Rs), t=np.stack(ts))

    # LineFilter (line_filter.py:12-21), identity at sigma=0.1 (Q13).
    pts = syn.room_scan((0.3, -0.2, 0.1), 180, seed=77, scan=0)
    sig = np.array([0.1, 0.2, 0.5, 1.0, 2.0, 3.7])
    outs = np.stack([LineFilter.filter(pts, sigma=s) for s in sig])
    short = rng.normal(0, 1, (5, 2))
    outs_short = np.stack([LineFilter.filter(short, sigma=s) for s in sig])
    np.savez_compressed(os.path.join(HERE, "unit_linefilter.npz"), points=pts, sigma=sig,
                        out=outs, short=short, out_short=outs_short)

    # Normalise / N_eff / resample / estimate on hand-made weight vectors.
    vecs = [np.array([1e-6, .5, .3, .1]), np.full(10, 1e-7), np.array([.2, .2, .2, .2, .2]),
            rng.random(37) ** 4, np.concatenate([rng.random(20) * 1e-5, rng.random(5)]),
            rng.random(64) * 3.0, np.array([0.0, 0.0, 1.0, 0.0])]
    recs = []
    for v in vecs:
        N = len(v)
        configure(N)
        fs = FastSLAM2()
        for i, p in enumerate(fs.particles):
            p.weight = float(v[i])
            p.x = float(i)
        wn = fs._FastSLAM2__normalize_weights()
        ne = fs._FastSLAM2__calculate_effective_particles()
        u0 = float(rng.uniform(0, 1.0 / N))
        saved = np.random.uniform
        np.random.uniform = lambda lo, hi, _u=u0: _u
        signal.signal(signal.SIGALRM, _alarm)
        signal.alarm(10)
        try:
            fs._FastSLAM2__low_variance_resample()
            src = np.array([int(p.x) for p in fs.particles])
        except Hang:
            src = np.full(N, -1)
        finally:
            signal.alarm(0)
            np.random.uniform = saved
        est = fs._FastSLAM2__estimate_robot_position()
        recs.append((v, wn, ne, u0, src, est[0]))
    np.savez_compressed(
        os.path.join(HERE, "unit_weights.npz"),
        **{f"w{k}": r[0] for k, r in enumerate(recs)},
        **{f"wn{k}": r[1] for k, r in enumerate(recs)},
        **{f"src{k}": r[4] for k, r in enumerate(recs)},
        n_eff=np.array([r[2] for r in recs]), u0=np.array([r[3] for r in recs]),
        est_index=np.array([r[5] for r in recs]), count=len(recs))
    print("units written")


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference not present: fixtures are committed, nothing to do")
    gen_units()
    gen_sequences()
