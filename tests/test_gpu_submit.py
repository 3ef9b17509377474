"""fs2_iterate_submit / fs2_iterate_wait (FastSLAM2.step_submit / step_wait).

The split call runs exactly the scan fs2_iterate runs (reference
fast_slam_2.py:33-67): same poses, stats, associations and state as a handle
stepped with step(); while a scan is pending the handle refuses any state
access (FS2_ERR_STATE), and a wait without a submission fails the same way
(two scans in flight: tests/test_gpu_pipelined.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_submit_wait_equals_step():
    import fast_slam_2
    import fs2_synthetic as syn
    from fast_slam_2 import _native as nat
    from gpu_util import configure
    configure()
    N, L = 20000, 60
    wl = syn.Workload(N, L, seed=9)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    lm[:, :, 2] = lm[:, :, 5] = 0.01
    hs = [fast_slam_2.FastSLAM2(N, rng="device", seed=4, record_assoc=True, landmark_capacity=L + 40,
                                verbose=False) for _ in range(2)]
    for h in hs:
        h.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
    resamples = 0
    for s in range(8):
        rot, tr = syn.odometry(s)
        ms = wl.measurements(s)
        p0, s0 = hs[0].step(rot, tr, ms)
        hs[1].step_submit(rot, tr, ms)
        with pytest.raises(nat.FS2Error):
            hs[1].associations()                      # (a second submit is allowed: test_gpu_pipelined.py)
        with pytest.raises(nat.FS2Error):
            hs[1].get_state(0, 4)                     # state is not readable mid-scan
        p1, s1 = hs[1].step_wait()
        assert np.array_equal(p0, p1), s
        assert s0.resampled == s1.resampled and s0.best_index == s1.best_index and s0.n_eff == s1.n_eff, s
        assert np.array_equal(hs[0].associations(), hs[1].associations()), s
        resamples += s0.resampled
    with pytest.raises(nat.FS2Error):
        hs[1].step_wait()                             # nothing pending
    a, b = hs[0].get_state(lm_cap=L + 40), hs[1].get_state(lm_cap=L + 40)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
    assert resamples >= 1
    for h in hs:
        h.close()
