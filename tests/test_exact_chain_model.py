"""CPU model of fs2_exact.hip's chain algorithm (binade translations + serial
units), checked against the sequential running sum on the stress cases of
test_gpu_exact.py.  This pins the algorithm's arithmetic argument on the host;
the GPU kernels are pinned against the C oracle by test_gpu_exact.py."""
import math

import numpy as np

UNIT = 64


def model_chain(a):
    n = len(a)
    nb = (n + 255) // 256
    bsum = np.array([a[b * 256:(b + 1) * 256].sum() for b in range(nb)])   # any order
    bpre = np.concatenate([[0.0], np.cumsum(bsum)[:-1]])
    margin = math.ldexp(2.0 * n + 8192.0, -53)
    nu = (n + UNIT - 1) // UNIT
    info, delta = [], []
    for k in range(nu):
        seg = a[k * UNIT:(k + 1) * UNIT]
        b = k // 4
        e_in = bpre[b] + sum(a[b * 256 + q * UNIT:b * 256 + (q + 1) * UNIT].sum() for q in range(k % 4))
        e_out = e_in + seg.sum()
        lo, hi = e_in * (1 - margin), e_out * (1 + margin)
        serial = k == 0 or not np.all((seg >= 0) & np.isfinite(seg)) or not (lo >= 2.0 ** -1020) \
            or not (hi < 2.0 ** 1020)
        E = 0
        if not serial:
            E = math.frexp(lo)[1] - 1
            serial = (math.frexp(hi)[1] - 1) != E
        D = 0
        if not serial:
            q = np.ldexp(seg, 52 - E)
            serial = bool(np.any(q - np.floor(q) == 0.5))
            D = int(np.rint(q).astype(np.int64).sum())
        info.append((serial, E))
        delta.append(0 if serial else D)
    c = np.empty(n)
    s = 0.0
    prev = -1
    for k in range(nu):
        serial, E = info[k]
        if not serial:
            continue
        if prev >= 0 and k > prev + 1:
            d = sum(delta[prev + 1:k])
            s = s + float(d) * math.ldexp(1.0, info[prev + 1][1] - 52)
        for j in range(k * UNIT, min(n, (k + 1) * UNIT)):
            s = a[j] if j == 0 else s + a[j]
            c[j] = s
        sin = s
        # translation units after k
        kk = k + 1
        while kk < nu and not info[kk][0]:
            E2 = info[kk][1]
            u = math.ldexp(1.0, E2 - 52)
            r = np.rint(np.ldexp(a[kk * UNIT:(kk + 1) * UNIT], 52 - E2)).astype(np.int64)
            pre = np.cumsum(r)
            c[kk * UNIT:kk * UNIT + len(r)] = sin + pre.astype(np.float64) * u
            sin = sin + float(pre[-1]) * u
            kk += 1
        prev = k
    return c


def test_chain_model_matches_running_sum():
    rng = np.random.default_rng(2024)
    N = 20_011
    cases = [rng.random(N) ** 6, rng.lognormal(0, 2, N), rng.random(N) * 1e-9]
    w = np.full(N, 2.0 ** -20 + 2.0 ** -54)
    w[5] = 0.5
    cases.append(w)
    w = rng.random(N)
    w[:1000] = 0.0
    cases.append(w)
    for a in cases:
        c = model_chain(a)
        assert np.array_equal(c, np.cumsum(a))
