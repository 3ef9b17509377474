"""CPU checks of the device draw of numpy's legacy RandomState (fs2_mt_draw,
fs2_mtrng.hpp), which replaces the reference's np.random.normal / uniform calls
(fast_slam_2/algorithms/fast_slam_2.py:79,81,183) in the drop-in iterate():

- the double-double log and its midpoint flag (the same host/device code, run on
  the CPU through fs2_debug_mt_log): every unflagged result equals libm's log
  (what numpy's legacy_gauss calls) bit for bit;
- a numpy restatement of the device algorithm (word recurrence in steps of 227,
  polar attempts ranked by a prefix count, output pairs, state after the draw and
  after u0) reproduces np.random.normal / uniform and np.random.get_state exactly,
  so the kernels' indexing is pinned against numpy itself before the GPU test
  (tests/test_gpu_mtrng.py) compares the device output."""
import ctypes as C
import math

import numpy as np
import pytest

from fast_slam_2 import _native as nat

MT_N, MT_LAG = 624, 227


def stream_words(key, total):
    """x[0..total): x[0..624) = key, x[n] = x[n-227] ^ twist(x[n-624], x[n-623])."""
    x = np.zeros(max(total, MT_N), dtype=np.uint32)
    x[:MT_N] = key
    n = MT_N
    while n < total:
        k = min(MT_LAG, total - n)
        j = np.arange(n, n + k)
        y = (x[j - 624] & np.uint32(0x80000000)) | (x[j - 623] & np.uint32(0x7fffffff))
        x[j] = x[j - 227] ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(0x9908b0df), np.uint32(0))
        n += k
    return x


def temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9d2c5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xefc60000))
    return y ^ (y >> np.uint32(18))


def legacy_double(w0, w1):
    a = (w0 >> np.uint32(5)).astype(np.float64)
    b = (w1 >> np.uint32(6)).astype(np.float64)
    return (a * 67108864.0 + b) / 9007199254740992.0


def model_draw(state, N, sigma):
    """The device draw restated: (noise[N], state after, state after u0, u0)."""
    _, key, pos, has_gauss, gauss = state
    h0 = 1 if (N > 0 and has_gauss) else 0
    P = (N - h0 + 1) // 2 if N > h0 else 0
    A = int(P / (math.pi / 4) + 12 * math.sqrt(P * (1 - math.pi / 4)) / (math.pi / 4)) + 64 if P else 0
    need = pos + 4 * A + 2
    total = max(MT_N, -(-need // MT_N) * MT_N)
    x = stream_words(np.asarray(key, dtype=np.uint32), total)
    t = temper(x[pos:pos + 4 * A].reshape(-1, 4)) if A else np.zeros((0, 4), np.uint32)
    x1 = 2.0 * legacy_double(t[:, 0], t[:, 1]) - 1.0
    x2 = 2.0 * legacy_double(t[:, 2], t[:, 3]) - 1.0
    r2 = x1 * x1 + x2 * x2
    ok = (r2 < 1.0) & (r2 != 0.0)
    acc = np.flatnonzero(ok)[:P]
    assert len(acc) == P
    out = np.empty(N)
    if h0:
        out[0] = 0.0 + sigma * gauss
    g_last = 0.0
    for r, a in enumerate(acc):
        f = math.sqrt(-2.0 * math.log(r2[a]) / r2[a])
        o = h0 + 2 * r
        out[o] = 0.0 + sigma * (f * x2[a])
        if o + 1 < N:
            out[o + 1] = 0.0 + sigma * (f * x1[a])
        else:
            g_last = f * x1[a]
    E = pos + 4 * (int(acc[-1]) + 1) if P else pos

    def at(e):
        if e == pos:
            return key, pos
        b = (e - 1) // MT_N
        return x[MT_N * b:MT_N * (b + 1)], e - MT_N * b

    if N == 0:
        hg, g = has_gauss, gauss
    elif P == 0:
        hg, g = 0, 0.0
    else:
        hg = 1 if (N - h0) % 2 else 0
        g = g_last if hg else 0.0
    k1, p1 = at(E)
    k2, p2 = at(E + 2)
    w = temper(x[E:E + 2])
    u0 = 0.0 + (1.0 / N - 0.0) * legacy_double(w[0:1], w[1:2])[0] if N else None
    return out, ("MT19937", k1, p1, hg, g), ("MT19937", k2, p2, hg, g), u0


def states_equal(a, b):
    return a[0] == b[0] and np.array_equal(np.asarray(a[1]), np.asarray(b[1])) and a[2] == b[2] \
        and a[3] == b[3] and a[4] == b[4]


def test_dd_log_unflagged_results_equal_libm():
    lib = nat.load()
    rs = np.random.RandomState(5)
    x = np.concatenate([rs.random_sample(60000) * rs.random_sample(60000), rs.random_sample(30000),
                        1.0 - rs.random_sample(10000) * 1e-9, [2.0 ** -104, 0.5, 0.25, np.nextafter(1.0, 0.0)]])
    x = x[(x > 0) & (x < 1)]
    out = np.empty_like(x)
    amb = np.empty(len(x), np.int32)
    nat.check(lib.fs2_debug_mt_log(0, nat.ptr(x), len(x), nat.ptr(out), nat.ptr(amb), 1))
    ref = np.array([math.log(v) for v in x])
    free = amb == 0
    assert np.array_equal(out[free], ref[free])
    # the flagged band is 2 x 0.025 ulp wide (plus powers of two)
    assert 0.03 < 1 - free.mean() < 0.07
    # and unflagged results are the double nearest the double-double value: every
    # flagged one is within one ulp of libm's
    assert np.all(np.abs(out[~free] - ref[~free]) <= np.spacing(np.abs(ref[~free])))


@pytest.mark.parametrize("seed,N,pre", [(0, 1, 0), (1, 2, 0), (2, 7, 1), (3, 1000, 0), (4, 1001, 3),
                                        (5, 20000, 0), (6, 0, 1), (7, 1, 1), (8, 4096, 5)])
def test_model_reproduces_numpy(seed, N, pre):
    """The restated device algorithm equals numpy's legacy stream, including an odd
    number of normals before (a cached gauss) and a state whose pos is mid-block."""
    np.random.seed(seed)
    np.random.normal(size=pre)
    np.random.random_sample(seed % 3)        # shift pos by words
    st = np.random.get_state()
    sigma = 0.0055
    noise, after, after_u0, u0 = model_draw(st, N, sigma)
    np.random.set_state(st)
    ref = np.random.normal(0, sigma, size=N)
    assert np.array_equal(noise, ref)
    assert states_equal(np.random.get_state(), after)
    if N:
        ru = np.random.uniform(0, 1 / N)
        assert ru == u0
        assert states_equal(np.random.get_state(), after_u0)


def test_mt_state_struct_round_trip():
    np.random.seed(11)
    np.random.normal(size=3)
    st = np.random.get_state()
    s = nat.fs2_mt_state.from_numpy(st)
    assert states_equal(s.to_numpy(), st)


@pytest.mark.parametrize("J", [1, 623, 624, 5000, 123457, 2600000])
def test_jump_ahead_words(J):
    """x[J + 1 .. J + 624] from the key by the jump polynomial (Berlekamp-Massey's
    characteristic polynomial, x^J mod it) equal the sequential stream's."""
    lib = nat.load()
    rs = np.random.RandomState(J % 1000)
    key = rs.randint(0, 2 ** 32, size=624, dtype=np.uint64).astype(np.uint32)
    out = np.zeros(624, dtype=np.uint32)
    nat.check(lib.fs2_debug_mt_jump(nat.ptr(key), J, nat.ptr(out)))
    ref = stream_words(key, J + 625)[J + 1:J + 625]
    assert np.array_equal(out, ref)
