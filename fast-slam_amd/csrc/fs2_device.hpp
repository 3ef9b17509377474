// fs2_device.hpp -- device math for the FastSLAM 2.0 hot path (gfx950, fp64).
//
// Operation order follows the reference (cy-rae/fast-slam) as executed by
// numpy 2.2 / OpenBLAS 0.3.29; where numpy delegates to BLAS/LAPACK the FMA
// placement was identified empirically and is restated with explicit fma()
// (the translation unit is compiled with -ffp-contract=off):
//   2x2 @ 2x2 (gemm)  C[i][j] = fma(A[i][1], B[1][j], A[i][0]*B[0][j])
//   2x2 @ vec (gemv)  r[i]    = fma(A[i][0], v[0],    A[i][1]*v[1])
//   vec @ 2x2         r[j]    = fma(v[1],   A[1][j],  v[0]*A[0][j])
//   dot               s       = fma(a[1],   b[1],     a[0]*b[0])
//   np.linalg.inv     LAPACK dgesv, partial pivoting, reciprocal scaling.
// This makes the association gate bit-identical to the reference.
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fs2 {

constexpr double kPi = 3.141592653589793;         // np.pi
constexpr double kTwoPi = 6.283185307179586;      // 2 * np.pi
constexpr double kLog2Pi = 1.8378770664093453;    // scipy _LOG_2PI = np.log(2 * np.pi)

// Python/numpy float floor-mod (numpy npy_divmod), b > 0 here.
__device__ __forceinline__ double pymod(double a, double b) {
    double m = fmod(a, b);
    if (m != 0.0) {
        if ((b < 0.0) != (m < 0.0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}

struct M2 {
    double a00, a01, a10, a11;
};

__device__ __forceinline__ M2 mm2(const M2 &A, const M2 &B) {
    M2 C;
    C.a00 = fma(A.a01, B.a10, A.a00 * B.a00);
    C.a01 = fma(A.a01, B.a11, A.a00 * B.a01);
    C.a10 = fma(A.a11, B.a10, A.a10 * B.a00);
    C.a11 = fma(A.a11, B.a11, A.a10 * B.a01);
    return C;
}

__device__ __forceinline__ M2 tr2(const M2 &A) { return M2{A.a00, A.a10, A.a01, A.a11}; }

// np.linalg.inv (2x2) -- see header comment.  Returns false when U is exactly
// singular (numpy raises LinAlgError).
__device__ __forceinline__ bool inv2(const M2 &A, M2 &out) {
    double r00 = A.a00, r01 = A.a01, r10 = A.a10, r11 = A.a11;
    const bool p = fabs(A.a10) > fabs(A.a00);
    if (p) {
        r00 = A.a10; r01 = A.a11; r10 = A.a00; r11 = A.a01;
    }
    if (r00 == 0.0) return false;
    const double ir00 = 1.0 / r00;
    const double l = r10 * ir00;
    const double u11 = r11 - l * r01;
    if (u11 == 0.0) return false;
    const double iu11 = 1.0 / u11;
    // column 0: b = P e0 ; column 1: b = P e1
    const double b00 = p ? 0.0 : 1.0, b01 = p ? 1.0 : 0.0;   // column 0 (b0, b1)
    const double b10 = p ? 1.0 : 0.0, b11 = p ? 0.0 : 1.0;   // column 1 (b0, b1)
    {
        const double y0 = b00, y1 = b01 - l * y0;
        const double x1 = y1 * iu11;
        out.a10 = x1;
        out.a00 = fma(-r01, x1, y0) * ir00;
    }
    {
        const double y0 = b10, y1 = b11 - l * y0;
        const double x1 = y1 * iu11;
        out.a11 = x1;
        out.a01 = fma(-r01, x1, y0) * ir00;
    }
    return true;
}

// delta^T inv delta with numpy's (vec @ 2x2) @ vec order (geometry_utils.py:22).
__device__ __forceinline__ double quad(const M2 &I, double d0, double d1) {
    const double r0 = fma(d1, I.a10, d0 * I.a00);
    const double r1 = fma(d1, I.a11, d0 * I.a01);
    return fma(r1, d1, r0 * d0);
}

// One landmark slot: mean and full (possibly asymmetric) covariance.
struct Slot {
    double mx, my;
    M2 P;
};

struct Meas {
    double d, b, ox, oy;
};

// ----------------------------------------------------------- gate mirror ---
// Every slot carries an fp32 shadow (x, y, s) read by the association pass in
// place of the 48-byte fp64 slot.  s is a lower bound on the smallest
// eigenvalue of the symmetric part of inv(P) -- the very inverse the gate uses
// (inv2) -- shrunk by 1e-6, so for the fp64 gate value q of ANY observed point
//     q >= s * |delta|^2.
// A slot whose fp32 lower bound on s*|delta|^2 (rounding of every fp32
// quantity accounted for, see gate_reject) exceeds gate2 can therefore not
// match, and is skipped without reading its fp64 data; every other slot takes
// the exact fp64 test.  Association results are unchanged by construction.
// s = 0 (never reject) when inv(P) is singular, not positive definite, not
// finite or worse conditioned than 1e8 (the 1e-6 margin covers the fp64
// rounding of q up to that condition number).
__device__ __forceinline__ float4 mirror_of(const Slot &sl) {
    M2 I;
    float s = 0.0f;
    if (inv2(sl.P, I)) {
        const double a = I.a00, c = I.a11, b = 0.5 * (I.a01 + I.a10);
        const double half = 0.5 * (a + c);
        const double dd = 0.5 * (a - c);
        const double lmax = half + sqrt(dd * dd + b * b);
        const double det = a * c - b * b;
        const double lmin = det / lmax;
        if (lmin > 0.0 && lmax < 1e300 && lmax <= 1e8 * lmin)
            s = __double2float_rd(lmin * (1.0 - 1e-6));
    }
    return make_float4(__double2float_rn(sl.mx), __double2float_rn(sl.my), s, 0.0f);
}

// A mirror's z holds s with its 12 low mantissa bits replaced by the slot's
// index in the map: pages may hold their 8 slots in any order (a map is laid
// out spatially at import), and the index keeps the reference's
// list order.  The bits are cleared before s is used, which only lowers it, so
// it stays a lower bound.
constexpr uint32_t kSlotBits = 0xfffu;        // slot indices < kMaxSlots = 4096
__device__ __forceinline__ float mirror_s(const float4 &m) {
    return __uint_as_float(__float_as_uint(m.z) & ~kSlotBits);
}
__device__ __forceinline__ int mirror_slot(const float4 &m) { return (int)(__float_as_uint(m.z) & kSlotBits); }
__device__ __forceinline__ float4 with_slot(float4 m, int slot) {
    m.z = __uint_as_float((__float_as_uint(m.z) & ~kSlotBits) | ((uint32_t)slot & kSlotBits));
    return m;
}

// true when the mirror proves sqrt(q) >= gate for the observed point (fx, fy).
//   |true dx| >= |fp32 dx| - ex,  ex = fe + (|x_lm| + |fp32 dx|) 2^-22
// (fe bounds the fp32 rounding of the observed point; the rounding of x_lm and
// of the subtraction is <= 2^-24 |value| each, so 2^-22 leaves a 4x margin).
// cx = 2^-22 |x_lm| and cy are per slot.  gate2f = gate2 / (1 - 2^-18) rounded
// up: the relative slack absorbs the fp32 rounding of lx, ly, d2 and s * d2.
__device__ __forceinline__ bool gate_reject_fast(const float4 &m, float cx, float cy, float fx,
                                                 float fy, float fe, float gate2f) {
    const float dx = fx - m.x, dy = fy - m.y;
    const float lx = fmaxf(fmaf(fabsf(dx), 0.99999976f, -(fe + cx)), 0.0f);
    const float ly = fmaxf(fmaf(fabsf(dy), 0.99999976f, -(fe + cy)), 0.0f);
    return mirror_s(m) * fmaf(lx, lx, ly * ly) > gate2f;
}

// EKF landmark update + likelihood (fast_slam_2.py:116-159).  Out of line: it
// runs a few times per particle and scan, and inlined at k_update's three call
// sites it would inflate the kernel's register footprint.
struct EkfOut {
    Slot s;
    double lik;
    int singular;
};

// Arguments and result by value, so that the call passes everything in VGPRs
// (a Slot& would live in scratch memory, and a scratch store ahead of the
// caller's next global load makes that load's wait cover the store too).
static __device__ __noinline__ EkfOut ekf_step(Slot s, double px, double py, double pyaw, double md,
                                              double mb, double r00, double r01, double r10, double r11) {
    const double dx = s.mx - px, dy = s.my - py;
    const double q = dx * dx + dy * dy;          // reference: pow(dx, 2) + pow(dy, 2)
    const double r = sqrt(q);
    const double ang = atan2(dy, dx) - pyaw;
    const double nu0 = md - r;
    const double nu1 = pymod((mb - ang) + kPi, kTwoPi) - kPi;
    const M2 H{dx / r, dy / r, -dy / q, dx / q};
    const M2 Ht = tr2(H);
    M2 S = mm2(mm2(H, s.P), Ht);
    S.a00 += r00; S.a01 += r01; S.a10 += r10; S.a11 += r11;
    M2 Si;
    if (!inv2(S, Si)) return EkfOut{s, 0.0, 1};
    const M2 K = mm2(mm2(s.P, Ht), Si);
    const double kn0 = fma(K.a00, nu0, K.a01 * nu1);
    const double kn1 = fma(K.a10, nu0, K.a11 * nu1);
    const M2 KH = mm2(K, H);
    const M2 IKH{1.0 - KH.a00, 0.0 - KH.a01, 0.0 - KH.a10, 1.0 - KH.a11};
    const M2 Pn = mm2(IKH, s.P);
    EkfOut o;
    o.s.mx = s.mx + kn0;
    o.s.my = s.my + kn1;
    o.s.P = Pn;
    // scipy: eigh on the lower triangle; closed form of log|S| and nu^T S^-1 nu.
    const double a = S.a00, b = S.a10, c = S.a11;
    const double det = a * c - b * b;
    const double maha = (c * nu0 * nu0 - 2.0 * b * nu0 * nu1 + a * nu1 * nu1) / det;
    o.lik = exp(-0.5 * (2.0 * kLog2Pi + log(det) + maha));
    o.singular = 0;
    return o;
}

// Updates `s` in place and returns the scipy multivariate_normal.pdf value.
__device__ __forceinline__ double ekf_update(Slot &s, double px, double py, double pyaw, const Meas &m,
                                             const M2 &R, bool &singular) {
    const EkfOut o = ekf_step(s, px, py, pyaw, m.d, m.b, R.a00, R.a01, R.a10, R.a11);
    if (o.singular) {
        singular = true;
        return 0.0;
    }
    s = o.s;
    return o.lik;
}

// ------------------------------------------------------------- Philox4x32-10
struct U4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// Uniform in (0, 1] from 53 random bits.
__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
    const uint64_t v = (((uint64_t)hi << 21) ^ (uint64_t)(lo >> 11)) & ((1ull << 53) - 1);
    return ((double)v + 1.0) * (1.0 / 9007199254740992.0);
}

// Standard normal for (stream, index) via Box-Muller on one Philox block.
__device__ __forceinline__ double philox_normal(uint64_t seed, uint64_t stream, uint64_t idx) {
    const U4 r = philox(U4{(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)stream,
                           (uint32_t)(stream >> 32)},
                        (uint32_t)seed, (uint32_t)(seed >> 32));
    const double u1 = u53(r.x, r.y), u2 = u53(r.z, r.w);
    return sqrt(-2.0 * log(u1)) * cos(kTwoPi * u2);
}

__device__ __forceinline__ double philox_uniform01(uint64_t seed, uint64_t stream, uint64_t idx) {
    const U4 r = philox(U4{(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)stream,
                           (uint32_t)(stream >> 32)},
                        (uint32_t)seed, (uint32_t)(seed >> 32));
    return u53(r.x, r.y) - (1.0 / 9007199254740992.0);   // [0, 1)
}

}  // namespace fs2
