"""Weights whose resample running sum (fast_slam_2.py:184-193) sits within the
exact chain's estimate margin of 2^0 for long stretches (fs2_exact.hip
k_chain_units): heavy weights normalise to a prefix just below 1, then groups of
small undivided weights (below the 1e-5 floor, Q6) walk it into the margin zone,
across 1 while still inside it, out of it, and on.  Between the groups a long
run of tiny weights: identity units (each term below half an ulp) whose estimate
straddles 2^0 -- on both sides of the crossing, so the binade their run is in
differs from the one the estimate's lower bound names and must be inherited."""
import numpy as np


def margin(n):
    """k_chain_units' relative bound for a chain of n terms (fs2_api.hip chain())."""
    return (2.0 * n + 8192.0) * 2.0 ** -53


def straddle_runs(N, rng, normalised=False):
    """Raw weights (or, with normalised, the chain's terms directly: the heavy
    pair already sums to the same prefix)."""
    d = margin(N) / 2.2
    w = 10.0 ** rng.uniform(-24, -18, N)
    S = 11.0 * d
    if normalised:
        w[10], w[20] = 0.5, 0.5 - S / 2        # prefix 1 - S/2
    else:
        w[10], w[20] = 1.2, 0.8                # normalise to ~0.6 + 0.4 = 1 - S/2 (total 2 + S)
    w[100:140] = 0.1 * d                       # into the zone: 1 - d/2 ... 1 - 1.5 d
    w[N // 5] = 2.0 * d                        # across 1, still inside: 1 + d/2
    w[3 * N // 10:3 * N // 10 + 40] = 0.1 * d  # out of it: 1 + 4.5 d
    w[7 * N // 10:7 * N // 10 + 10] = 0.1 * d  # translations with D != 0 after identities
    return w
