// fs2_plan.hpp -- the arithmetic of the low-variance resample plan (reference
// fast_slam_2/algorithms/fast_slam_2.py:177-199), shared by the device kernels
// (fs2_resample.hip: k_ranges, k_pack_*) and the host entry points fs2_plan_*
// (include/fs2.h) that tests/test_dist_plan.py runs per rank on the CPU.  Both
// are compiled with -ffp-contract=off, so host and device round alike.
//
// With u_m = u0 + m * (1/N) evaluated as the reference writes it and c the
// inclusive prefix of the normalised weights, global particle g fills the
// contiguous outputs { m : c_{g-1} < u_m <= c_g } (particle N-1 also every m
// with u_m > c_{N-2}, where the reference would loop forever).  The
// ranges are non-decreasing in g, so the local particles whose outputs reach
// rank p's shard are one run of the local index (empty ranges aside).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fs2 {

__host__ __device__ inline double plan_u(double u0, int64_t m, int64_t N) {
    return u0 + (double)m * (1.0 / (double)N);      // fast_slam_2.py:189, as written
}

// first output m in [0, N] with u_m > v.  u_m is non-decreasing in m (the
// rounded product and sum are monotone), so the answer is unique: start from
// the real-arithmetic estimate and step to it (a step or two at most, bounded
// by a binary search fallback).
__host__ __device__ inline int64_t plan_first_above(double v, double u0, int64_t N) {
    // a NaN prefix: `u > NaN` is false for every u, so the reference's loop stops
    // at the particle whose running sum turned NaN and it fills every later output
    if (v != v) return N;
    const double est = (v - u0) * (double)N;
    int64_t m = (est < 0.0) ? 0 : (est >= (double)N ? N : (int64_t)est + 1);
    for (int it = 0; it < 8; ++it) {
        if (m > 0 && plan_u(u0, m - 1, N) > v) --m;
        else if (m < N && !(plan_u(u0, m, N) > v)) ++m;
        else return m;
    }
    int64_t lo = 0, hi = N;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (plan_u(u0, mid, N) > v) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// Output range [lo, hi] (empty when lo > hi) of global particle g whose prefix
// before it is prev and through it cur.
__host__ __device__ inline void plan_range(int64_t g, int64_t N, double prev, double cur, double u0, int64_t &lo,
                                           int64_t &hi) {
    lo = (g == 0) ? 0 : plan_first_above(prev, u0, N);
    hi = (g == N - 1) ? N - 1 : plan_first_above(cur, u0, N) - 1;
}

// Rank p's shard [N p / G, N (p + 1) / G) of particles and of outputs.
__host__ __device__ inline int64_t shard_begin(int64_t N, int G, int p) { return N * p / G; }

// A non-empty range [lo, hi] that reaches shard [pa, pb).
__host__ __device__ inline bool plan_reaches(int64_t lo, int64_t hi, int64_t pa, int64_t pb) {
    return lo <= hi && lo < pb && hi >= pa;
}

// First index i in [0, n) with key(i) >= v for a non-decreasing key (n if none).
template <typename K>
__host__ __device__ inline int64_t plan_lower_bound(int64_t n, int64_t v, K key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (key(mid) >= v) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// The run [i0, i1) of local particles whose outputs may reach shard [pa, pb):
// every non-empty range inside it reaches the shard and none outside does
// (mhi and mlo are non-decreasing in the local index).
template <typename LO, typename HI>
__host__ __device__ inline void plan_run(int64_t n, int64_t pa, int64_t pb, LO mlo, HI mhi, int64_t &i0,
                                         int64_t &i1) {
    i0 = plan_lower_bound(n, pa, mhi);
    i1 = plan_lower_bound(n, pb, mlo);
    if (i1 < i0) i1 = i0;
}

}  // namespace fs2
