// fs2_mtrng.hpp -- numpy's legacy RandomState (MT19937 + the polar Gaussian) as
// host/device arithmetic, for the drop-in FastSLAM2.iterate() draws:
//   fast_slam_2.py:79,81   np.random.normal(0, ROTATION_NOISE / TRANSLATION_NOISE)
//   fast_slam_2.py:183     np.random.uniform(0, 1 / NUM_PARTICLES)
// numpy (numpy/random/src/mt19937, src/legacy/legacy-distributions.c):
//   mt19937_next: a 624-word state twisted in place, each output tempered;
//   legacy_double: (a >> 5, b >> 6) of two outputs -> (a 2^26 + b) / 2^53;
//   legacy_gauss: cached second value, else x1 = 2 d - 1, x2 = 2 d - 1 until
//     0 < r2 = x1 x1 + x2 x2 < 1, f = sqrt(-2 log(r2) / r2), cache f x1, return f x2;
//   legacy_normal(loc, scale) = loc + scale * legacy_gauss.
// The word stream is the linear recurrence x[n] = x[n-227] ^ twist(x[n-624], x[n-623])
// (the in-place twist of the 624-word key restated over the stream), so one
// workgroup generates 227 words per step, two steps per barrier pair (fs2_mtrng.hip).  Everything but log(r2) is
// exact or correctly rounded (IEEE mul / add / div / sqrt), identical on host and
// device; log is glibc's (error <= 0.52 ulp, not always correctly rounded), so the
// device evaluates log in double-double and flags the results within 0.025 ulp of
// a rounding midpoint, which the host recomputes with libm's log.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <cmath>

namespace fs2 {

constexpr int kMtN = 624, kMtM = 397;
constexpr int kMtLag = kMtN - kMtM;        // 227: words one step of the recurrence yields
constexpr uint32_t kMtMatrixA = 0x9908b0dfu, kMtUpper = 0x80000000u, kMtLower = 0x7fffffffu;
constexpr double kMtAmbBand = 0.025;        // ulps around a midpoint the host recomputes

__host__ __device__ inline uint32_t mt_next_word(uint32_t x_n624, uint32_t x_n623, uint32_t x_n227) {
    const uint32_t y = (x_n624 & kMtUpper) | (x_n623 & kMtLower);
    return x_n227 ^ (y >> 1) ^ ((y & 1u) ? kMtMatrixA : 0u);
}

__host__ __device__ inline uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// legacy_double of two tempered outputs (exact)
__host__ __device__ inline double mt_double(uint32_t w0, uint32_t w1) {
    const int32_t a = (int32_t)(w0 >> 5), b = (int32_t)(w1 >> 6);
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

// One polar attempt from four raw (untempered) stream words.
struct MtAttempt {
    double x1, x2, r2;
    bool ok;
};
__host__ __device__ inline MtAttempt mt_attempt(uint32_t r0, uint32_t r1, uint32_t r2w, uint32_t r3) {
    MtAttempt a;
    a.x1 = 2.0 * mt_double(mt_temper(r0), mt_temper(r1)) - 1.0;
    a.x2 = 2.0 * mt_double(mt_temper(r2w), mt_temper(r3)) - 1.0;
    const double p1 = a.x1 * a.x1, p2 = a.x2 * a.x2;   // separate roundings (no fma), as numpy's build
    a.r2 = p1 + p2;
    a.ok = a.r2 < 1.0 && a.r2 != 0.0;
    return a;
}

// ---- double-double arithmetic (every product / sum written out: no contraction) ----
struct DD {
    double hi, lo;
};
__host__ __device__ inline uint64_t dbits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
__host__ __device__ inline double dfrom(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}
__host__ __device__ inline DD dd_two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return DD{s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline DD dd_fast(double a, double b) {   // |a| >= |b|
    const double s = a + b;
    return DD{s, b - (s - a)};
}
__host__ __device__ inline DD dd_two_prod(double a, double b) {
    const double p = a * b;
#ifdef __HIP_DEVICE_COMPILE__
    return DD{p, __builtin_fma(a, b, -p)};
#else
    return DD{p, std::fma(a, b, -p)};
#endif
}
__host__ __device__ inline DD dd_add(DD a, DD b) {
    DD s = dd_two_sum(a.hi, b.hi);
    const DD t = dd_two_sum(a.lo, b.lo);
    s.lo = s.lo + t.hi;
    s = dd_fast(s.hi, s.lo);
    s.lo = s.lo + t.lo;
    return dd_fast(s.hi, s.lo);
}
__host__ __device__ inline DD dd_mul(DD a, DD b) {
    DD p = dd_two_prod(a.hi, b.hi);
    const double c1 = a.hi * b.lo, c2 = a.lo * b.hi;
    p.lo = p.lo + (c1 + c2);
    return dd_fast(p.hi, p.lo);
}
__host__ __device__ inline DD dd_mul_d(DD a, double b) {
    DD p = dd_two_prod(a.hi, b);
    const double c = a.lo * b;
    p.lo = p.lo + c;
    return dd_fast(p.hi, p.lo);
}
__host__ __device__ inline DD dd_div(DD a, DD b) {
    const double q1 = a.hi / b.hi;
    DD r = dd_add(a, dd_mul_d(b, -q1));
    const double q2 = r.hi / b.hi;
    r = dd_add(r, dd_mul_d(b, -q2));
    const double q3 = r.hi / b.hi;
    return dd_add(dd_fast(q1, q2), DD{q3, 0.0});
}
// 1 / k as a double-double (the division's remainder is exact)
__host__ __device__ inline DD dd_inv(double k) {
    const double h = 1.0 / k;
    DD p = dd_two_prod(h, k);                 // h k = 1 - e exactly (p.hi + p.lo)
    const double e = (1.0 - p.hi) - p.lo;
    return DD{h, e / k};
}

// log(x) for a positive normal x as a double-double (relative error ~2^-100):
// x = 2^e m, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m - 1) / (m + 1),
// |s| <= 0.1716, the series sum_j s^(2j+1) / (2j+1) to j = 21 (s^44 / 45 < 2^-107).
constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
__host__ __device__ inline DD dd_log(double x) {
    const uint64_t u = dbits(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023;
    double m = dfrom((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);   // [1, 2)
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e += 1;
    }
    const DD num{m - 1.0, 0.0};               // exact (Sterbenz)
    const DD s = dd_div(num, dd_two_sum(m, 1.0));
    const DD t = dd_mul(s, s);
    DD p = dd_inv(43.0);
#pragma unroll
    for (int j = 20; j >= 0; --j) p = dd_add(dd_mul(t, p), dd_inv(2.0 * j + 1.0));
    const DD lm = dd_mul(dd_mul_d(s, 2.0), p);
    const double ed = (double)e;
    const DD kl = dd_add(dd_two_prod(ed, kLn2Hi), DD{ed * kLn2Lo, 0.0});
    return dd_add(kl, lm);
}

// The table form used per draw: x = 2^e m, m in [0.75, 1.5), c = 1 + i/128 the
// nearest table point (i in [-32, 64]; m - c exact), log m = log c + 2 atanh(s),
// s = (m - c) / (m + c), |s| <= 1/512, seven series terms (s^16 / 15 < 2^-140).
// c = 1 exactly around m = 1, so a result near 0 (r2 near 1) cancels nothing.
// log c (double-double) comes from dd_log; host and device compute the same table
// bit for bit (IEEE operations and exact fma only).
constexpr int kMtLogTab = 97;
__host__ __device__ inline DD mt_log_tab_entry(int k) {
    const double c = 1.0 + (double)(k - 32) / 128.0;
    return (k == 32) ? DD{0.0, 0.0} : dd_log(c);
}
__host__ __device__ inline DD dd_log_tab(double x, const double *thi, const double *tlo) {
    const uint64_t u = dbits(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023;
    double m = dfrom((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);   // [1, 2)
    if (m >= 1.5) {
        m = m * 0.5;
        e += 1;
    }
#ifdef __HIP_DEVICE_COMPILE__
    const double fi = __builtin_rint((m - 1.0) * 128.0);
#else
    const double fi = std::rint((m - 1.0) * 128.0);
#endif
    const int k = (int)fi + 32;
    const double c = 1.0 + fi / 128.0;
    const DD s = dd_div(DD{m - c, 0.0}, dd_two_sum(m, c));
    const DD t = dd_mul(s, s);
    DD p = dd_inv(15.0);
#pragma unroll
    for (int j = 6; j >= 0; --j) p = dd_add(dd_mul(t, p), dd_inv(2.0 * j + 1.0));
    const DD lm = dd_add(DD{thi[k], tlo[k]}, dd_mul(dd_mul_d(s, 2.0), p));
    const double ed = (double)e;
    const DD kl = dd_add(dd_two_prod(ed, kLn2Hi), DD{ed * kLn2Lo, 0.0});
    return dd_add(kl, lm);
}

// log(x) rounded to double, and whether the rounding is not certain to equal
// glibc's (the double-double value lies within kMtAmbBand ulp of a midpoint, or
// the result is a power of two, where the ulp changes).  x in (0, 1).
__host__ __device__ inline double mt_log(double x, const double *thi, const double *tlo, bool *amb) {
    const DD l = dd_log_tab(x, thi, tlo);
    const uint64_t au = dbits(l.hi) & 0x7fffffffffffffffull;
    const int ex = (int)(au >> 52);
    const double ulp = dfrom((uint64_t)(ex - 52) << 52);
    const double frac = fabs(l.lo) / ulp;
    *amb = frac > 0.5 - kMtAmbBand || (au & 0x000fffffffffffffull) == 0 || ex < 53;
    return l.hi;
}

// f = sqrt(-2 log(r2) / r2) with a given log
__host__ __device__ inline double mt_polar_f(double r2, double lg) {
    const double num = -2.0 * lg;
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_sqrt(num / r2);
#else
    return std::sqrt(num / r2);
#endif
}

}  // namespace fs2
