"""The in-place view of numpy's global legacy RandomState used by the drop-in
iterate() (fast_slam_2/_npstate.py) against numpy's own get_state / set_state:
states with and without a cached gauss, pos anywhere in the block, reseeds."""
import ctypes as C

import numpy as np
import pytest


def test_view_reads_and_writes_what_numpy_does():
    from fast_slam_2 import _native as nat
    from fast_slam_2 import _npstate
    v = _npstate.view()
    if v is None:
        pytest.skip("this numpy's RandomState layout is not the proven one (get_state / set_state used)")
    rng = np.random.default_rng(3)
    for trial in range(40):
        np.random.seed(int(rng.integers(0, 2**31)))
        np.random.random_sample(int(rng.integers(0, 700)))
        np.random.normal(size=int(rng.integers(0, 3)))        # odd: a cached gauss
        st = np.random.get_state()
        got = nat.fs2_mt_state()
        v.read(got)
        assert np.array_equal(np.frombuffer(bytes(got.key), np.uint32), st[1])
        assert (got.pos, got.has_gauss, got.gauss) == (st[2], st[3], st[4])
        # write another state; numpy's draws continue from it
        np.random.seed(trial)
        np.random.normal(size=trial % 3)
        other = np.random.get_state()
        ref = np.random.normal(size=5)
        np.random.set_state(st)
        w = nat.fs2_mt_state.from_numpy(other)
        v.write(w)
        back = np.random.get_state()
        assert np.array_equal(back[1], other[1]) and back[2:] == other[2:]
        assert np.array_equal(np.random.normal(size=5), ref)


def test_view_follows_a_reseed():
    from fast_slam_2 import _native as nat
    from fast_slam_2 import _npstate
    v = _npstate.view()
    if v is None:
        pytest.skip("layout not recognised")
    np.random.seed(11)
    a = nat.fs2_mt_state()
    _npstate.view().read(a)
    np.random.seed(12)
    b = nat.fs2_mt_state()
    _npstate.view().read(b)
    assert bytes(a.key) != bytes(b.key)
    assert np.array_equal(np.frombuffer(bytes(b.key), np.uint32), np.random.get_state()[1])
