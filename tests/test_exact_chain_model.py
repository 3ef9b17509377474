"""CPU model of fs2_exact.hip's chain algorithm (binade translations + serial
units), checked against the sequential running sum on the stress cases of
test_gpu_exact.py.  This pins the algorithm's arithmetic argument on the host;
the GPU kernels are pinned against the C oracle by test_gpu_exact.py."""
import math

import numpy as np

UNIT = 64


def model_chain(a, return_units=False):
    """fs2_exact.hip: k_chain_units (per-term binade estimates -> one translation,
    up to 4 segments, or term by term), k_chain_walk and its prefix post-pass."""
    n = len(a)
    nb = (n + 255) // 256
    bsum = np.array([a[b * 256:(b + 1) * 256].sum() for b in range(nb)])   # any order
    bpre = np.concatenate([[0.0], np.cumsum(bsum)[:-1]])
    margin = math.ldexp(2.0 * n + 8192.0, -53)
    nu = (n + UNIT - 1) // UNIT
    units = []
    for k in range(nu):
        seg = a[k * UNIT:(k + 1) * UNIT]
        b = k // 4
        e_in = bpre[b] + sum(a[b * 256 + q * UNIT:b * 256 + (q + 1) * UNIT].sum() for q in range(k % 4))
        incl = e_in + np.cumsum(seg)
        lo, hi = (incl - seg) * (1 - margin), incl * (1 + margin)
        ok, okt, E, r = [], [], [], []
        for j, v in enumerate(seg):
            base = k * UNIT + j != 0 and 0 <= v < np.inf and lo[j] >= 2.0 ** -1020 and hi[j] < 2.0 ** 1020
            e = math.frexp(lo[j])[1] - 1 if base else -4096
            o = base and math.frexp(hi[j])[1] - 1 == e
            # (round 6) below half the step of binade e: an identity in e and above
            ident = base and not o and math.ldexp(v, 52 - e) < 0.5
            rr = 0
            if o:
                q = math.ldexp(v, 52 - e)
                o = q - math.floor(q) != 0.5
                rr = int(np.rint(q)) if o else 0
            okt.append(o)
            ok.append(o or ident)
            E.append(e)
            r.append(rr)
        if all(okt) and len(set(E)) == 1:
            units.append(("t", E[0], sum(r)))
            continue
        if all(o and rr == 0 for o, rr in zip(ok, r)):
            # (round 6) every term an identity: a translation by 0 whose binade is
            # inherited (the estimate may straddle a boundary the chain never crosses)
            units.append(("i", E[0], 0))
            continue
        segs = []
        for j in range(len(seg)):
            if j == 0 or not ok[j] or not ok[j - 1] or E[j] != E[j - 1]:
                segs.append([j, j + 1])
            else:
                segs[-1][1] = j + 1
        if len(segs) > 8:
            units.append(("w", None, None))
            continue
        desc = []
        for st, en in segs:
            if ok[st]:
                desc.append(("t", E[st], sum(r[st:en]), st, en))
            else:
                desc.append(("s", None, seg[st], st, en))
        units.append(("g", desc, None))
    # Elast(k): the binade of the last translation unit proper at or before k (identity
    # units inherit it; None: no such unit, so every run before k adds 0)
    elast, e = [], None
    for kind, x, y in units:
        if kind == "t":
            e = x
        elast.append(e)
    c = np.empty(n)
    s_out, dsum = 0.0, 0               # value after the last listed unit, D since it
    for k, (kind, x, y) in enumerate(units):
        lo_i = k * UNIT
        vals = a[lo_i:lo_i + UNIT]
        er = elast[k - 1] if k > 0 else None
        assert dsum == 0 or er is not None
        s_in = s_out + float(dsum) * (math.ldexp(1.0, er - 52) if er is not None else 0.0)
        if kind in "ti":
            if kind == "i":
                c[lo_i:lo_i + len(vals)] = s_in
            else:
                u = math.ldexp(1.0, x - 52)
                pre = np.cumsum(np.rint(np.ldexp(vals, 52 - x)).astype(np.int64))
                c[lo_i:lo_i + len(vals)] = s_in + pre.astype(np.float64) * u
            dsum += y
            continue
        s = s_in
        if kind == "w":
            out, s = chain_unit_ref(vals, s, k == 0)
            c[lo_i:lo_i + len(vals)] = out
        else:
            for sk, e, d, st, en in x:
                if sk == "s":
                    c[lo_i + st] = s + d
                    s = s + d
                else:
                    u = math.ldexp(1.0, e - 52)
                    pre = np.cumsum(np.rint(np.ldexp(vals[st:en], 52 - e)).astype(np.int64))
                    c[lo_i + st:lo_i + en] = s + pre.astype(np.float64) * u
                    s = s + float(d) * u
        s_out, dsum = s, 0
    return (c, units, elast) if return_units else c


def chain_unit_ref(vals, s, first):
    out = np.empty(len(vals))
    for j, v in enumerate(vals):
        s = v if (first and j == 0) else s + v
        out[j] = s
    return out, s


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
    # (round 6) a chain that reaches 1 - 6e-11 early, then only tiny terms: the
    # estimate's margin straddles 2^0 for every later term (identities, one segment
    # per unit instead of a term-by-term walk); also heavy terms after such a stretch
    w = 10.0 ** rng.uniform(-23, -8, N)
    w[100] = 1.0 - 6.5e-11 - w[:100].sum()
    cases.append(w)
    w2 = w.copy()
    w2[15000] = 0.25
    cases.append(w2)
    for a in cases:
        c = model_chain(a)
        assert np.array_equal(c, np.cumsum(a))


def test_chain_model_identity_units_inherit_binade():
    """(round 6) chain_cases.straddle_runs: units of identities alone whose estimate
    straddles 2^0 are translations by 0 in the binade of the run they sit in --
    below 1 before the crossing, above it after, where the estimate's lower bound
    still names [0.5, 1)."""
    from chain_cases import straddle_runs
    a = straddle_runs(20011, np.random.default_rng(3), normalised=True)
    c, units, elast = model_chain(a, return_units=True)
    assert np.array_equal(c, np.cumsum(a))
    kinds = [u[0] for u in units]
    idx = [k for k, kd in enumerate(kinds) if kd == "i"]
    assert len(idx) > 50
    # identities after the crossing (chain in [1, 2)) still name [0.5, 1) ...
    cross = 20011 // 5 // 64
    after = [k for k in idx if k > cross and c[k * 64] >= 1.0]
    assert after and all(units[k][1] == -1 for k in after)
    # ... and translations with D != 0 follow in [1, 2)
    assert any(kd == "t" and units[k][1] == 0 and units[k][2] > 0 for k, kd in enumerate(kinds))


def model_chain_unit(a, s, first):
    """fs2_chain.hpp chain_unit: wave-wide steps inside one binade, one plain add
    at the first crossing / tie / bad term."""
    cnt = len(a)
    out = np.zeros(cnt)
    j0 = 0
    if first:
        s = a[0]
        out[0] = s
        j0 = 1
    while j0 < cnt:
        if s == 0.0:
            nz = [j for j in range(j0, cnt) if a[j] != 0.0]
            jn = nz[0] if nz else cnt
            out[j0:jn] = s
            if jn >= cnt:
                break
            s = s + a[jn]
            out[jn] = s
            j0 = jn + 1
            continue
        if not (2.0 ** -1020 <= s < 2.0 ** 1020):
            s = s + a[j0]
            out[j0] = s
            j0 += 1
            continue
        E = math.frexp(s)[1] - 1
        u, top = math.ldexp(1.0, E - 52), math.ldexp(1.0, E + 1)
        js, P = cnt, 0
        vals = {}
        for j in range(j0, cnt):
            with np.errstate(over="ignore"):
                q = float(np.ldexp(a[j], 52 - E))
            ok = a[j] >= 0 and q < 2.0 ** 53
            r = int(np.rint(q)) if ok else 0
            P += r
            v = s + float(P) * u
            if (not ok) or (q - math.floor(q) == 0.5 if ok else True) or v >= top:
                js = j
                break
            vals[j] = v
        for j, v in vals.items():
            out[j] = v
        if js >= cnt:
            s = vals[cnt - 1] if vals else s
            break
        sp = s if js == j0 else vals[js - 1]
        s = sp + a[js]
        out[js] = s
        j0 = js + 1
    return out, s


def test_chain_unit_model_matches_sequential():
    rng = np.random.default_rng(7)
    for trial in range(400):
        kind = trial % 5
        if kind == 0:
            a = rng.random(64) * 10.0 ** rng.uniform(-8, 0)
            s = float(rng.random() * 10.0 ** rng.uniform(-8, 1))
        elif kind == 1:                    # crossings inside the unit: s just below a power of 2
            s = math.ldexp(1.0, int(rng.integers(-20, 5))) * (1 - 1e-9)
            a = rng.random(64) * s * 1e-3
        elif kind == 2:                    # ties at [0.5, 1)
            s = 0.75
            a = np.full(64, 2.0 ** -20 + 2.0 ** -54)
        elif kind == 3:                    # zeros, then growth from 0
            s = 0.0
            a = np.where(rng.random(64) < 0.5, 0.0, rng.random(64) * 1e-300)
        else:                              # fast growth from a tiny start
            s = 1e-300
            a = 10.0 ** rng.uniform(-300, 2, 64)
        first = trial % 7 == 0
        got, send = model_chain_unit(a, s, first)
        ref = np.empty(64)
        t = s
        for j in range(64):
            t = a[j] if (first and j == 0) else t + a[j]
            ref[j] = t
        assert np.array_equal(got, ref), trial
        assert send == ref[-1]
