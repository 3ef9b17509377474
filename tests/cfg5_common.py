"""Inputs shared by the config-5-shape test and its rank processes
(tests/test_gpu_config5_shape.py, tests/cfg5_worker.py): one definition of the
initial scalars, the per-scan draws and the checks' sampling, so the parent's
oracle and the ranks see the same numbers."""
import numpy as np

WINDOW = 256


def CAP(L, scans):
    return L + 4 * scans + 8


def initial_scalars(N):
    """Poses of SURVEY §8d, weights of a filter some scans in (lognormal, spread
    enough that the N_eff < N/2 rule fires on some scans and not on others)."""
    import fs2_synthetic as syn
    x, y, yaw = syn.particle_poses(N, 0)
    wh = np.random.default_rng(77).lognormal(0.0, 0.85, N)
    return x, y, yaw, wh / wh.sum()


def draws(N, L, scans):
    """Per scan: odometry, measurements, the N motion normals and the
    resample start of the reference's draws (fast_slam_2.py:79,81,183)."""
    import fs2_synthetic as syn
    rng = np.random.default_rng(8)
    for s in range(scans):
        rot, tr = syn.odometry(s)
        ms = syn.scan_measurements(L, s, 0)
        nz = rng.normal(0, 0.001 if rot else 0.0055, N)
        u0 = rng.uniform(0, 1.0 / N)
        yield rot, tr, ms, nz, u0


def window_start(N, s):
    return int(np.random.default_rng(1000 + s).integers(0, N - WINDOW))


def map_checksum(lm):
    """One number per particle map [k][cap][6]: a weighted sum of every entry (the
    weights keep slots and fields apart), compared within a relative tolerance."""
    k, cap = lm.shape[0], lm.shape[1]
    wts = (1.0 + 1e-3 * np.arange(cap))[:, None] * np.array([1.0, 2.0, 3.0, 5.0, 7.0, 11.0])[None, :]
    return np.einsum("pcf,cf->p", lm, wts)
