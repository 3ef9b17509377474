"""The shard-policy replay of scripts/drift_study.py on
synthetic resampling histories (CPU): every policy's shards tile the global
order, the movable policy respects its cap and keeps at least as many outputs
local as equal shards following their sources, and nothing moves less than the
forced lower bound."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scripts"))


def _history(N, drift, rng):
    """out_src of a systematic resample whose normalised weights sum to `drift`
    (Q6 leaves small weights undivided): outputs come from the first N / drift sources."""
    w = rng.exponential(1.0, N) * (rng.random(N) < 0.6)
    c = np.cumsum(w / w.sum() * drift)
    u = (np.arange(N) + rng.random()) / N
    return np.minimum(np.searchsorted(c, u), N - 1)


@pytest.mark.parametrize("G,drift,cap", [(2, 1.4, 1.15), (4, 1.1, 1.15), (8, 1.37, 1.15), (8, 2.5, 1.25)])
def test_policies_tile_and_bound(G, drift, cap):
    import drift_study as ds
    rng = np.random.default_rng(G)
    N = 4096 * G
    starts, order = ds.equal_starts(N, G), list(range(G))
    for _ in range(3):
        src = _history(N, drift, rng)
        lo, hi = ds.natural(src, starts, order)
        assert lo[0] == 0 and hi[-1] == N and np.all(lo[1:] == hi[:-1])     # natural intervals tile [0, N)
        forced = int(np.maximum(0, (hi - lo) - int(cap * N / G)).sum())
        fs, fo = ds.follow(src, starts, order, N, G)
        ms, mo = ds.movable(src, starts, order, N, G, cap)
        for cuts, own in ((fs, fo), (ms, mo)):
            assert cuts[0] == 0 and cuts[-1] == N and np.all(np.diff(cuts) >= 0)
            assert sorted(own) == list(range(G))                          # every rank holds one interval
        assert np.diff(ms).max() <= cap * N / G + 1
        f_out = ds.moved(src, starts, fs, fo, order)[0]
        m_out = ds.moved(src, starts, ms, mo, order)[0]
        assert forced <= m_out
        # the DP cuts on a grid of N / (64 G): it may lose up to a unit per interval
        assert m_out <= f_out + G * (N // (64 * G) + 1)
        starts, order = ms, mo
