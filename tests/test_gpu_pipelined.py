"""Two scans submitted before the first is waited for (fs2.h fs2_iterate_submit):
the second submit completes the outstanding scan first and keeps its results for
the next fs2_iterate_wait, so results come back in submission order.  (Round 5
enqueued the second scan's update pass behind the first one's tail, reading its
buffer set on the device; measured no faster and removed in round 6.)  The
results must be the bits of step() one scan at a time -- reference semantics
fast_slam_2.py:33-223 -- on a workload that resamples often, with device Philox
draws and with injected noise / u0 (the pinned staging is per scan parity), and
with scans of two update passes (M > 4); a third outstanding submit is refused."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(N, L, seed, **kw):
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    wl = syn.Workload(N, L, seed=seed)
    x, y, yaw = wl.poses()
    lm = wl.maps()
    lm[:, :, 2] = lm[:, :, 5] = 0.01            # peaked likelihoods: frequent resamples
    hs = []
    for _ in range(2):
        f = fast_slam_2.FastSLAM2(N, rng="device", seed=9, landmark_capacity=L + 40, verbose=False, **kw)
        f.set_state(x, y, yaw, np.full(N, 1.0 / N), np.full(N, L, np.int32), lm)
        hs.append(f)
    return wl, hs


def _same(a, b):
    pa, sa = a
    pb, sb = b
    assert np.array_equal(pa, pb), (pa, pb)
    for k in ("resampled", "best_index", "n_eff", "total_weight", "hits", "appends", "cow_pages",
              "slots_visited", "error_flags"):
        assert getattr(sa, k) == getattr(sb, k), (k, getattr(sa, k), getattr(sb, k))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("inject", [False, True])
def test_two_in_flight_equals_one_at_a_time(inject):
    import fs2_synthetic as syn
    N, L, S = 120_000, 48, 14
    wl, (ref, pip) = _pair(N, L, 5)
    rng = np.random.default_rng(3)
    draws = [(rng.normal(0, 0.001, N), rng.uniform(0, 1.0 / N)) for _ in range(S)] if inject else [(None, None)] * S
    want = []
    for s in range(S):
        nz, u0 = draws[s]
        want.append(ref.step(*syn.odometry(s), wl.measurements(s), None, nz, u0))
    got = []
    for s in range(S):
        nz, u0 = draws[s]
        pip.step_submit(*syn.odometry(s), wl.measurements(s), None, nz, u0)
        if s > 0:
            got.append(pip.step_wait())
    got.append(pip.step_wait())
    assert sum(int(st.resampled) for _, st in want) >= 3
    for s in range(S):
        _same(got[s], want[s])
    a, b = ref.get_state(lm_cap=L + 40), pip.get_state(lm_cap=L + 40)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
    ref.close()
    pip.close()


@pytest.mark.timeout(300)
def test_non_overlapping_scan_completes_the_outstanding_one():
    """Eight measurements (two update passes) on every third scan: the results come
    back in submission order and equal step()'s."""
    import fs2_synthetic as syn
    N, L, S = 60_000, 32, 8
    wl, (ref, pip) = _pair(N, L, 7)

    def meas(s):
        m = wl.measurements(s)
        return np.vstack([m, m]) if s % 3 == 1 else m
    want = [ref.step(*syn.odometry(s), meas(s)) for s in range(S)]
    got = []
    for s in range(S):
        pip.step_submit(*syn.odometry(s), meas(s))
        if s > 0:
            got.append(pip.step_wait())
    got.append(pip.step_wait())
    for s in range(S):
        _same(got[s], want[s])
    with pytest.raises(Exception):
        pip.step_wait()                          # nothing outstanding
    ref.close()
    pip.close()


@pytest.mark.timeout(120)
def test_three_outstanding_scans_are_refused():
    import fs2_synthetic as syn
    from fast_slam_2._native import FS2Error
    N, L = 20_000, 16
    wl, (a, b) = _pair(N, L, 2)
    b.close()
    a.step_submit(*syn.odometry(0), wl.measurements(0))
    a.step_submit(*syn.odometry(1), wl.measurements(1))
    with pytest.raises(FS2Error):
        a.step_submit(*syn.odometry(2), wl.measurements(2))
    with pytest.raises(FS2Error):
        a.step(*syn.odometry(2), wl.measurements(2))      # step() needs nothing outstanding
    a.step_wait()
    a.step_wait()
    a.step(*syn.odometry(2), wl.measurements(2))
    a.close()
