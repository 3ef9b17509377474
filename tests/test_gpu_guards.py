"""No kernel writes past the end of a buffer (FS2_GUARD=1: fs2_create follows
every buffer with a 64 KiB pattern, fs2_debug_check_guards names the first one
whose pattern changed).  Round 6 found k_normalize_chunks writing one partial per
half numpy chunk into a buffer sized per chunk: silent at N = 1e6 (inside the
allocation's granule), a memory fault at N = 8e6.  The scans below cover every
reduction mode (sequential, parallel, exact with and without the chunked
normalisation), resampling scans (the prefix, range and gather kernels), appends,
collections and particle counts that are not multiples of the block sizes."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(f):
    from fast_slam_2 import _native as nat
    name = C.create_string_buffer(128)
    bad = nat.load().fs2_debug_check_guards(f._h, name, 128)
    assert bad == 0, f"{bad} guard bytes overwritten after buffer {name.value.decode()}"


@pytest.mark.timeout(300)
@pytest.mark.parametrize("N,L,reduce,scans", [(100, 20, "auto", 6), (20011, 50, "parallel", 6),
                                               (100_003, 200, "auto", 8), (1_000_000, 500, "auto", 8),
                                               (2_500_000, 60, "auto", 6)])
def test_no_write_past_a_buffer(N, L, reduce, scans):
    import torch  # noqa: F401  -- (bench.populate fills the maps on the GPU)
    import bench
    import fast_slam_2
    import fs2_synthetic as syn
    from gpu_util import configure
    configure()
    old = os.environ.get("FS2_GUARD")
    os.environ["FS2_GUARD"] = "1"
    try:
        f = fast_slam_2.FastSLAM2(N, rng="device", seed=3, reduce=reduce, landmark_capacity=L + 4 * scans + 8,
                                  verbose=False)
    finally:
        if old is None:
            os.environ.pop("FS2_GUARD", None)
        else:
            os.environ["FS2_GUARD"] = old
    bench.populate(f, N, L, 0, 0)
    _check(f)
    res = 0
    for s in range(scans):
        _, st = f.step(*syn.odometry(s), np.ascontiguousarray(syn.scan_measurements(L, s, 0)))
        res += st.resampled
        _check(f)
    f.close()
    if N >= 100_000:
        assert res >= 1
