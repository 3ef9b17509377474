"""The reference's summation orders on large N (fs2_exact.hip, FS2_REDUCE_EXACT).

The reference normalises with Python's sum (fast_slam_2.py:166), resamples along
a running sum built one particle at a time (:184-193) and takes N_eff from
np.sum(w ** 2) (:219-223).  In EXACT mode (the default on one GPU above 4096
particles) libfs2 evaluates those orders with parallel kernels and must agree
with the C oracle's sequential loops bit for bit: the weight total, every
normalised weight, N_eff, the decision and every resample source.  The cases
stress what the parallel evaluation has to get right: many binades crossed,
exact rounding ties (round-half-even depends on the running value), leading
zeros, a u_m landing exactly on a prefix value, N_eff exactly N/2, all-zero and
subnormal weights (one exact grid below 2^-1021).  The tree
mode (PARALLEL) reports such near-boundary decisions in reduce_ambiguous.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fs():
    import torch  # noqa: F401
    import fast_slam_2
    yield fast_slam_2


def seq_sum(a):
    t = 0.0
    for v in a.tolist():
        t += v
    return t


def seq_prefix(a):
    return np.cumsum(a)          # numpy's cumsum is the sequential running sum


def expected(w, u0):
    from oracle import oracle as orc
    wn = orc.normalize(w)
    ne = orc.n_eff(wn)
    N = len(w)
    rs = ne < N / 2.0
    src = orc.resample_src(wn, u0) if rs else np.arange(N)
    return seq_sum(w), wn, ne, rs, src


def run_tail(fs, w, u0, reduce, with_pose=False):
    """One scan without measurements and without motion: only the tail
    (normalise, N_eff, resample, estimate) changes the state; x = particle index
    reveals each output's source."""
    N = len(w)
    f = fs.FastSLAM2(N, reduce=reduce, verbose=False)
    f.set_state(np.arange(N, dtype=float), np.zeros(N), np.zeros(N), w)
    pose, st = f.step(0.0, 0.0, np.zeros((0, 2)), None, np.zeros(N), u0)
    x, _, _, wn, _, _ = f.get_state()
    f.close()
    if with_pose:
        return st, x.astype(np.int64), wn, pose
    return st, x.astype(np.int64), wn


def expected_estimate(wn, src):
    """fast_slam_2.py:201-210 after the resample: Python's max over the particles by
    weight, the first of equal ones; x of output m is its source's index."""
    ow = wn[src]
    return float(src[int(np.argmax(ow))])


def cases():
    rng = np.random.default_rng(2024)
    out = []
    N = 100_003
    out.append(("binades", rng.random(N) ** 6, 0.37 / N))
    # ties: 2^-20 + 2^-54 is an odd multiple of half the ulp of [0.5, 1); the big
    # weight makes the normalised prefix live there (the small ones stay
    # un-divided below the 1e-5 floor)
    w = np.full(N, 2.0 ** -20 + 2.0 ** -54)
    w[5] = 0.5
    out.append(("ties", w, 0.61 / N))
    w = rng.random(N)
    w[:1000] = 0.0
    out.append(("leading_zeros", w * 1e-3, 0.5 / N))
    # u_0 exactly equal to the prefix value c_7 (u > c is false there)
    w = rng.random(N) * 1e-9
    w[10] = 3.0
    c = seq_prefix(w)
    out.append(("u_on_boundary", w, float(c[7])))
    # N_eff exactly N / 2: half the weights 2/N, half 0 (not < N/2: no resample)
    M = 65_536
    w = np.zeros(M)
    w[::2] = 2.0 / M
    out.append(("neff_half", w, 0.5 / M))
    out.append(("full_chunks", rng.random(3 * 8192) ** 3, 0.2 / (3 * 8192)))
    # partial last chunks of 3 (under numpy's 8-element block), 100 (one leaf) and
    # 8191 (the deepest tree) elements
    for tail in (3, 100, 8191):
        n = 2 * 8192 + tail
        out.append((f"tail_{tail}", rng.random(n) ** 2, 0.3 / n))
    out.append(("cfg3_size", rng.lognormal(0.0, 2.0, 1_000_000), 0.77e-6))
    # the heaviest particle receives no output: the undivided weights below 1e-5 (Q6)
    # sum past 1 before it, so the post-resample estimate is another particle's
    n = 200_003
    w = np.full(n, 9e-6)
    w[150_000] = 0.01
    out.append(("heavy_unsampled", w, 0.4 / n))
    # equal heaviest weights far apart: the estimate is the first one's first output
    w = rng.random(n) * 1e-7
    w[70_001] = w[20_000] = 0.25
    out.append(("estimate_tie", w, 0.3 / n))
    # a diverged filter: every likelihood underflowed (the total is 0, the
    # reference resets the weights to 1/N) -- the chain runs on zeros throughout
    out.append(("all_zero", np.zeros(1_000_000), 0.5e-6))
    # the grid below 2^-1021 (subnormals, zeros) and the crossing out of it into
    # the normal binades, then into the weights that normalise
    w = rng.integers(0, 1 << 40, 200_003).astype(np.float64) * 2.0 ** -1074
    w[::7] = 0.0
    w[120_000:] = rng.random(80_003) * 1e-300
    w[190_000:] = rng.random(10_003) * 1e-3
    out.append(("subnormal_grid", w, 0.45 / 200_003))
    # (round 6) the normalised chain reaches 1 - ~1e-10 after two heavy weights, then
    # a million tiny ones: the prefix estimate's margin straddles 2^0 for every later
    # term (identities, listed as one segment per unit; the appended-maps workload's
    # 2.5 ms walk), and both heavy sources take >100 K outputs (k_fill_runs)
    w = 10.0 ** rng.uniform(-24, -15, 1_000_000)
    w[10], w[20] = 0.3, 0.2
    out.append(("straddle_one", w, 0.3e-6))
    # (round 6) identity units on both sides of a crossing inside the margin zone
    # (translations by 0 whose binade is inherited, tests/chain_cases.py)
    from chain_cases import straddle_runs
    out.append(("straddle_runs", straddle_runs(1_000_000, rng), 0.7e-6))
    return out


@pytest.mark.parametrize("name,w,u0", cases(), ids=[c[0] for c in cases()])
def test_exact_tail_matches_reference_order(fs, name, w, u0):
    total, wn, ne, rs, src = expected(w, u0)
    st, xs, wg, pose = run_tail(fs, w, u0, "exact", with_pose=True)
    assert st.total_weight == total, name
    assert np.array_equal(wg, wn[src]), name
    assert st.n_eff == ne, name
    assert bool(st.resampled) == rs, name
    assert np.array_equal(xs, src), name
    assert st.reduce_ambiguous == 0
    # the estimate (published before the resample's gather on one GPU)
    assert pose[0] == expected_estimate(wn, src), name


@pytest.mark.parametrize("reduce,n", [("sequential", 3001), ("parallel", 150_000)])
def test_post_resample_estimate_other_modes(fs, reduce, n):
    """The same estimate rule in the sequential and the tree reduction modes: at
    3001 particles two equal heaviest weights (the first one's first output); at
    150 000 the heaviest particle left without an output (the undivided weights
    below 1e-5 pass 1 before it)."""
    w = np.full(n, 9e-6)
    w[(3 * n) // 4] = 0.01
    if n < 10_000:
        w[n // 3] = 0.01
    w[n // 8] = w[n // 5] = 3e-6    # below 1e-5, undivided (lighter than the rest)
    u0 = 0.45 / n
    total, wn, ne, rs, src = expected(w, u0)
    assert rs
    st, xs, _, pose = run_tail(fs, w, u0, reduce, with_pose=True)
    # (tree sums: boundaries within the rounding bound may go the other way, and
    # are counted; the estimate is checked on the resample that ran)
    assert np.array_equal(xs, src) or (reduce == "parallel" and st.reduce_ambiguous > 0)
    assert pose[0] == expected_estimate(wn, xs)


def test_auto_is_exact_above_4096(fs):
    w = np.random.default_rng(5).random(50_000) ** 4
    u0 = 0.3 / 50_000
    total, wn, ne, rs, src = expected(w, u0)
    st, xs, _ = run_tail(fs, w, u0, "auto")
    assert st.total_weight == total and st.n_eff == ne
    assert np.array_equal(xs, src)


def test_tree_mode_reports_boundary_ties(fs):
    """PARALLEL (tree) sums: a u_m exactly on a prefix value and N_eff exactly N/2
    are reported as ambiguous; EXACT mode resolves both like the reference."""
    name, w, u0 = [c for c in cases() if c[0] == "u_on_boundary"][0]
    st, xs, _ = run_tail(fs, w, u0, "parallel")
    assert st.resampled == 1 and st.reduce_ambiguous >= 1
    name, w, u0 = [c for c in cases() if c[0] == "neff_half"][0]
    st, _, _ = run_tail(fs, w, u0, "parallel")
    assert st.reduce_ambiguous >= 1
    st, _, _ = run_tail(fs, w, u0, "exact")
    assert st.reduce_ambiguous == 0 and st.resampled == 0
