// fs2_exact.hip -- the reference's summation orders, evaluated in parallel and
// bit-exactly on gfx950.
//
// Three reductions of the per-scan tail depend on the order the reference sums in:
//   * the weight total, Python's builtin sum over the particles
//     (fast_slam_2.py:166): s_0 = w_0, s_k = fl(s_{k-1} + w_k);
//   * the resample's running sum (fast_slam_2.py:184-193), the same chain over
//     the normalised weights, compared against u_m at every step;
//   * np.sum(weights ** 2) (fast_slam_2.py:219-223): numpy's pairwise sum inside
//     8192-element buffer chunks, the chunk sums added in order.
// A fixed-order tree gives values a few ulps off the reference's, so a
// resample boundary near some u_m can pick a different source.  The kernels
// below reproduce the reference's values exactly, in parallel:
//
// Chain (sum and prefix).  All terms are >= 0, so the chain is non-decreasing
// and passes through each binade [2^(E), 2^(E+1)) at most once.  While the
// running value s stays inside one binade its grid is u = 2^(E-52), s is a
// multiple of u, and (no ties) fl(s + a) = s + rint(a / u) u exactly.  So a
// 64-element unit whose chain values provably stay in one binade is a pure
// translation by D u, D = sum of rint(a_k / u) (an exact int64 sum, any order);
// the binade test uses a tree estimate of the prefix with the rigorous bound
// |s_k - R_k| <= k 2^-53 R_k of recursive summation (R: the exact prefix)
// doubled.  Units that may cross a binade, hold a tie (a / u an odd multiple
// of 1/2: fl rounds to even, which depends on s), a non-finite or negative
// term, or the chain's first element are evaluated one add at a time.  Only
// those (~20-40 per chain: one per binade crossed) are walked serially; the
// translations between them are an integer scan.
//
//   k_chain_bpre   exclusive prefix of the 256-element block sums (tree estimate)
//   k_chain_units  per unit: translation (binade E, D) or serial
//   k_chain_walk   one workgroup: integer scan of D, then the serial units in
//                  order (wave 0, the 64 terms of a unit broadcast lane by lane)
//   k_chain_fill   prefix mode: each translation unit's values s_in + (scan of
//                  rint(a/u)) u
//
// numpy sum of squares.  Each full 8192-element chunk is numpy's pairwise tree:
// 64 leaves of 128 elements (8 accumulators of 16 sequential adds, combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))), the leaves combined as a balanced
// binary tree in order -- one wave per chunk, xor butterflies.  A partial last
// chunk is summed by lane 0 with the recursive form.  The chunk sums are added
// in order by k_finalize.
#include "fs2_reduce.hpp"

namespace fs2 {

constexpr int kUnit = 64;                  // chain unit: one wave
constexpr int kNpChunk = 8192;             // numpy's reduction buffer

__device__ __forceinline__ bool lazy_skip(const ChainParams &P) {
    return P.stats != nullptr && !P.stats->resampled;
}

__device__ __forceinline__ double bcast(double v, int j) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), j);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ long long wave_sum_i64(long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ long long wave_incl_scan_i64(long long v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// ulp of the binade E (values in [2^E, 2^(E+1))) and a / ulp rounded to nearest
__device__ __forceinline__ double unit_ulp(int E) { return ldexp(1.0, E - 52); }
__device__ __forceinline__ double scaled(double a, int E) { return ldexp(a, 52 - E); }

// --------------------------------------------------------------- chain ----

// Exclusive prefix of the block sums (one workgroup): estimates of the chain's
// value at every block start.
__global__ __launch_bounds__(1024) void k_chain_bpre(const ChainParams P) {
    __shared__ double lds[16];
    if (P.lazy && lazy_skip(P)) return;
    const int t = threadIdx.x;
    const int per = (P.nb + 1023) / 1024;
    const int b0 = t * per, b1 = min(P.nb, b0 + per);
    double run = 0.0;
    for (int b = b0; b < b1; ++b) run += P.bsum[b];
    // wave inclusive scan, then the waves before
    double incl = run;
    const int lane = t & 63, wid = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) lds[wid] = incl;
    __syncthreads();
    double off = incl - run;
    for (int k = 0; k < wid; ++k) off += lds[k];
    for (int b = b0; b < b1; ++b) {
        P.bpre[b] = off;
        off += P.bsum[b];
    }
}

// Per 64-element unit (one wave; 4 units per 256-element block): translation
// (info = (E + 4096) << 1, delta = D) or serial (info bit 0).
__global__ __launch_bounds__(kBlock) void k_chain_units(const ChainParams P) {
    __shared__ double s_ws[kBlock / 64];
    if (P.lazy && lazy_skip(P)) return;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int64_t i = (int64_t)blockIdx.x * kBlock + t;
    const int64_t k = (int64_t)blockIdx.x * (kBlock / kUnit) + wid;
    const int64_t nu = (P.n + kUnit - 1) / kUnit;
    const double a = (i < P.n) ? P.a[i] : 0.0;
    const bool bad = (i < P.n) && !(a >= 0.0 && a < INFINITY);
    const double us = wave_sum(a);
    if (lane == 0) s_ws[wid] = us;
    __syncthreads();
    if (k >= nu) return;
    double e_in = P.bpre[blockIdx.x];
    for (int q = 0; q < wid; ++q) e_in += s_ws[q];
    const double e_out = e_in + us;
    const double lo = e_in * (1.0 - P.margin), hi = e_out * (1.0 + P.margin);
    bool serial = (k == 0) || __any(bad) || !(lo >= 0x1p-1020) || !(hi < 0x1p1020);
    int E = 0;
    if (!serial) {
        E = ilogb(lo);
        serial = ilogb(hi) != E;
    }
    long long r = 0;
    if (!serial) {
        const double q = scaled(a, E);         // < 2^53: exact
        const double fq = floor(q);
        serial = __any(q - fq == 0.5);         // a tie: rounding depends on s
        r = (long long)rint(q);
    }
    const long long D = serial ? 0 : wave_sum_i64(r);
    if (lane == 0) {
        P.uinfo[k] = serial ? 1 : ((E + 4096) << 1);
        P.udelta[k] = D;
    }
}

// One workgroup: the integer scan over units, then wave 0 walks the serial
// units in order.  Writes the value after each serial unit (sout, by ordinal),
// the chain's values inside serial units (prefix mode) and the total.
__global__ __launch_bounds__(1024) void k_chain_walk(const ChainParams P) {
    __shared__ unsigned long long s_d[16];
    __shared__ int s_c[16];
    __shared__ int s_nseq;
    if (P.lazy && lazy_skip(P)) return;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int64_t nu = (P.n + kUnit - 1) / kUnit;
    if (nu == 0) {
        if (t == 0 && P.total) *P.total = 0.0;
        return;
    }
    const int64_t per = (nu + 1023) / 1024;
    const int64_t k0 = t * per, k1 = min(nu, k0 + per);
    unsigned long long ds = 0;
    int sc = 0;
    for (int64_t k = k0; k < k1; ++k) {
        ds += (unsigned long long)P.udelta[k];
        sc += P.uinfo[k] & 1;
    }
    // exclusive scans over threads (wrapping uint64: differences inside a run are exact)
    unsigned long long di = ds;
    int ci = sc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long v = __shfl_up(di, o, 64);
        const int c = __shfl_up(ci, o, 64);
        if (lane >= o) {
            di += v;
            ci += c;
        }
    }
    if (lane == 63) {
        s_d[wid] = di;
        s_c[wid] = ci;
    }
    __syncthreads();
    unsigned long long dx = di - ds;
    int cx = ci - sc;
    for (int q = 0; q < wid; ++q) {
        dx += s_d[q];
        cx += s_c[q];
    }
    if (t == 1023) s_nseq = cx + sc;
    for (int64_t k = k0; k < k1; ++k) {
        P.ug[k] = dx;
        dx += (unsigned long long)P.udelta[k];
        if (P.uinfo[k] & 1) P.seql[cx++] = (int32_t)k;
        P.uord[k] = cx - 1;
    }
    __syncthreads();
    if (wid != 0) return;
    __threadfence_block();
    const int nseq = s_nseq;
    double s = 0.0;
    int64_t prev = -1;
    // the next serial unit's terms are loaded one unit ahead
    auto load_unit = [&](int o) -> double {
        if (o >= nseq) return 0.0;
        const int64_t i = (int64_t)P.seql[o] * kUnit + lane;
        return i < P.n ? P.a[i] : 0.0;
    };
    double a = load_unit(0);
    for (int o = 0; o < nseq; ++o) {
        const int64_t q = P.seql[o];
        const double an = load_unit(o + 1);
        if (prev >= 0 && q > prev + 1) {       // translation run prev+1 .. q-1
            const int E = (P.uinfo[prev + 1] >> 1) - 4096;
            const long long d = (long long)(P.ug[q] - P.ug[prev + 1]);
            s = s + (double)d * unit_ulp(E);
        }
        const int cnt = (int)min<int64_t>(kUnit, P.n - q * kUnit);
        double mine = 0.0;
        for (int j = 0; j < cnt; ++j) {
            const double v = bcast(a, j);
            s = (q == 0 && j == 0) ? v : s + v;
            if (lane == j) mine = s;
        }
        if (P.c && lane < cnt) P.c[q * kUnit + lane] = mine;
        if (lane == 0) P.sout[o] = s;
        prev = q;
        a = an;
    }
    if (lane == 0 && P.total) {
        double tot = s;
        if (prev < nu - 1) {                    // the chain ends in a translation run
            const int E = (P.uinfo[prev + 1] >> 1) - 4096;
            const long long d = (long long)(P.ug[nu - 1] + (unsigned long long)P.udelta[nu - 1] - P.ug[prev + 1]);
            tot = s + (double)d * unit_ulp(E);
        }
        *P.total = tot;
    }
}

// Prefix mode: the chain's values inside translation units.
__global__ __launch_bounds__(kBlock) void k_chain_fill(const ChainParams P) {
    if (P.lazy && lazy_skip(P)) return;
    const int t = threadIdx.x, wid = t >> 6;
    const int64_t i = (int64_t)blockIdx.x * kBlock + t;
    const int64_t k = (int64_t)blockIdx.x * (kBlock / kUnit) + wid;
    const int64_t nu = (P.n + kUnit - 1) / kUnit;
    if (k >= nu) return;
    const int32_t info = P.uinfo[k];
    if (info & 1) return;                       // serial units were written by the walk
    const int E = (info >> 1) - 4096;
    const int o = P.uord[k];
    const int64_t q = P.seql[o];
    const double u = unit_ulp(E);
    const double s_in = P.sout[o] + (double)(long long)(P.ug[k] - P.ug[q + 1]) * u;
    const double a = (i < P.n) ? P.a[i] : 0.0;
    const long long pre = wave_incl_scan_i64((long long)rint(scaled(a, E)));
    if (i < P.n) P.c[i] = s_in + (double)pre * u;
}

hipError_t launch_chain(const ChainParams &p, hipStream_t s) {
    if (p.n <= 0) {
        if (p.total) hipLaunchKernelGGL(k_chain_walk, dim3(1), dim3(1024), 0, s, p);
        return hipGetLastError();
    }
    const unsigned nb = (unsigned)((p.n + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_chain_bpre, dim3(1), dim3(1024), 0, s, p);
    hipLaunchKernelGGL(k_chain_units, dim3(nb), dim3(kBlock), 0, s, p);
    hipLaunchKernelGGL(k_chain_walk, dim3(1), dim3(1024), 0, s, p);
    if (p.c) hipLaunchKernelGGL(k_chain_fill, dim3(nb), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------- numpy sum of w^2 --

// numpy pairwise summation of a[i]^2 (loops_utils.h.src: PW_BLOCKSIZE 128, 8
// accumulators), recursive form; used for a partial last chunk.
__device__ double np_pairwise_sq(const double *a, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; ++i) res += a[i] * a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = a[k] * a[k];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8) {
#pragma unroll
            for (int k = 0; k < 8; ++k) r[k] += a[i + k] * a[i + k];
        }
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i] * a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_sq(a, n2) + np_pairwise_sq(a + n2, n - n2);
}

// One wave per 8192-element chunk -> part[chunk].
__global__ __launch_bounds__(64) void k_np_sumsq(const double *w, int64_t n, double *part, const DevStats *lazy) {
    if (lazy && !lazy->resampled) return;
    const int lane = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * kNpChunk;
    const int64_t m = min<int64_t>(kNpChunk, n - c0);
    if (m < kNpChunk) {
        if (lane == 0) part[blockIdx.x] = np_pairwise_sq(w + c0, m);
        return;
    }
    // lane = 8 * g + k: accumulator k of leaf 8 * batch + g
    const int g = lane >> 3, k = lane & 7;
    double leaf = 0.0;                         // lane l ends up holding leaf l's sum
#pragma unroll 1
    for (int bt = 0; bt < 8; ++bt) {
        const double *p = w + c0 + (int64_t)(8 * bt + g) * 128 + k;
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = p[8 * q];
        double r = v[0] * v[0];
#pragma unroll
        for (int q = 1; q < 16; ++q) r += v[q] * v[q];
        r += __shfl_xor(r, 1, 64);             // (r0 + r1), (r2 + r3), ...
        r += __shfl_xor(r, 2, 64);             // ((r0 + r1) + (r2 + r3)), ...
        r += __shfl_xor(r, 4, 64);
        // leaf 8 * bt + g's sum sits in lanes 8g .. 8g+7; lane 8 bt + g takes it
        const double got = __shfl(r, 8 * ((lane - 8 * bt) & 7), 64);
        if ((lane >> 3) == bt) leaf = got;
    }
    // balanced tree over the 64 leaves in order
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) leaf += __shfl_xor(leaf, o, 64);
    if (lane == 0) part[blockIdx.x] = leaf;
}

hipError_t launch_np_sumsq(const double *w, int64_t n, double *part, const DevStats *lazy, hipStream_t s) {
    const int64_t nc = (n + kNpChunk - 1) / kNpChunk;
    if (nc == 0) return hipSuccess;
    hipLaunchKernelGGL(k_np_sumsq, dim3((unsigned)nc), dim3(64), 0, s, w, n, part, lazy);
    return hipGetLastError();
}

int64_t np_sumsq_chunks(int64_t n) { return (n + kNpChunk - 1) / kNpChunk; }

}  // namespace fs2
