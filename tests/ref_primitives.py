#!/usr/bin/env python3
"""Run the reference's hot-path primitives on a batch of inputs (test helper).

Used by tests/test_oracle_vs_reference.py, in a subprocess of its own because the
reference package is also called `fast_slam_2`.  Imports the reference from
/root/reference with empty HAL / cv2 stub modules, reads the
cases from an .npz and writes the reference's outputs to another .npz.  Only the
reference's outputs leave this process.

  python tests/ref_primitives.py cases.npz out.npz
"""
import signal
import sys
import types

import numpy as np

REF = "/root/reference"


class _Hang(Exception):
    pass


def _alarm(signum, frame):
    raise _Hang()


def main(inp, outp):
    sys.modules.setdefault("HAL", types.ModuleType("HAL"))
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, REF)
    import fast_slam_2.algorithms.fast_slam_2 as fs_mod
    from fast_slam_2 import ICP, GeometryUtils, Landmark, LandmarkUtils, LineFilter, Particle
    import fast_slam_2.utils.landmark_utils as lu_mod

    d = np.load(inp)
    out = {}
    # Mahalanobis distance (geometry_utils.py:13-23)
    out["maha"] = np.array([GeometryUtils.mahalanobis_distance(a, b, c)
                            for a, b, c in zip(d["maha_a"], d["maha_b"], d["maha_cov"])])
    # first-match association (landmark_utils.py:92-117)
    assoc = []
    for k in range(len(d["as_obs"])):
        L = int(d["as_len"][k])
        lms = [Landmark(float(x), float(y), c.reshape(2, 2).copy())
               for x, y, c in zip(d["as_lm"][k, :L, 0], d["as_lm"][k, :L, 1], d["as_lm"][k, :L, 2:6])]
        lu_mod.MAXIMUM_LANDMARK_DISTANCE = float(d["as_gate"][k])
        _, idx = LandmarkUtils.associate_landmarks(Landmark(*map(float, d["as_obs"][k])), lms)
        assoc.append(-1 if idx is None else idx)
    out["assoc"] = np.array(assoc)
    # weights: normalise, N_eff, estimate, low-variance resample (fast_slam_2.py:161-223)
    nw, ne, est, src = [], [], [], []
    signal.signal(signal.SIGALRM, _alarm)
    for k in range(len(d["w_len"])):
        N = int(d["w_len"][k])
        w = d["w"][k, :N]
        fs_mod.NUM_PARTICLES = N
        fs = fs_mod.FastSLAM2.__new__(fs_mod.FastSLAM2)
        fs.particles = []
        for i in range(N):
            p = Particle(float(i), 0.0, 0.0)     # x = original index, to identify copies
            p.weight = float(w[i])
            fs.particles.append(p)
        nwk = fs._FastSLAM2__normalize_weights()
        nw.append(np.pad(nwk, (0, d["w"].shape[1] - N)))
        ne.append(fs._FastSLAM2__calculate_effective_particles())
        est.append(fs._FastSLAM2__estimate_robot_position()[0])
        u0 = float(d["u0"][k])
        saved = np.random.uniform
        np.random.uniform = lambda lo, hi: u0
        signal.alarm(5)
        try:
            fs._FastSLAM2__low_variance_resample()
            s = [int(p.x) for p in fs.particles]
        except _Hang:
            s = [-2] * N                         # the reference hangs here
        finally:
            signal.alarm(0)
            np.random.uniform = saved
        src.append(np.pad(np.array(s), (0, d["w"].shape[1] - N), constant_values=-3))
    out["norm_w"], out["n_eff"], out["est_x"], out["src"] = np.array(nw), np.array(ne), np.array(est), np.array(src)
    # ICP best fit and full alignment (icp.py:13-90)
    R, t = zip(*[ICP.best_fit_transform(a, b) for a, b in zip(d["bf_src"], d["bf_tgt"])])
    out["bf_R"], out["bf_t"] = np.array(R), np.array(t)
    R, t = zip(*[ICP.get_transformation(a, b) for a, b in zip(d["icp_src"], d["icp_tgt"])])
    out["icp_R"], out["icp_t"] = np.array(R), np.array(t)
    # LineFilter (line_filter.py:12-21)
    out["lf"] = np.array([LineFilter.filter(p, sigma=float(s)) for p, s in zip(d["lf_pts"], d["lf_sigma"])])
    np.savez(outp, **out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
