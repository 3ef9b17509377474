// fs2_chain.hpp -- device helpers of the exact-order chain (fs2_exact.hip), shared
// with the resample's range kernel, which evaluates the running sum's values from
// the chain's unit table instead of reading a materialised prefix.
#pragma once

#include "fs2_reduce.hpp"

namespace fs2 {

constexpr int kUnit = 64;                  // chain unit: one wave

__device__ __forceinline__ double bcast(double v, int j) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), j);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ long long wave_sum_i64(long long v) {
    return lane63(dpp_scan(v, 0ll, [](long long a, long long b) { return a + b; }));
}

__device__ __forceinline__ long long wave_incl_scan_i64(long long v) {
    return dpp_scan(v, 0ll, [](long long a, long long b) { return a + b; });
}

// ulp of the binade E (values in [2^E, 2^(E+1))) and a / ulp
__device__ __forceinline__ double unit_ulp(int E) { return ldexp(1.0, E - 52); }
__device__ __forceinline__ double scaled(double a, int E) { return ldexp(a, 52 - E); }
__device__ __forceinline__ int unit_binade(int32_t info) { return (info >> 2) - 4096; }
// binade of a chain value v >= 0 whose grid the chain runs on: values below 2^-1021
// (zero, subnormals, [2^-1022, 2^-1021)) share the step 2^-1074 = unit_ulp(-1022)
__device__ __forceinline__ int chain_binade(double v) { return v < 0x1p-1021 ? -1022 : ilogb(v); }

__device__ __forceinline__ long long bcast_i64(long long v, int j) {
    return __double_as_longlong(bcast(__longlong_as_double(v), j));
}

__device__ __forceinline__ double wave_incl_scan_f64(double v) {
    return dpp_scan(v, 0.0, [](double a, double b) { return a + b; });
}

// Exclusive prefix of in[0..n) into out (1024 threads; a tree estimate).
__device__ inline void block_excl_scan_1024(const double *in, double *out, int n, double *lds16) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int per = (n + 1023) / 1024;
    const int b0 = min(n, t * per), b1 = min(n, b0 + per);
    double run = 0.0;
    for (int b = b0; b < b1; ++b) run += in[b];
    double incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    __syncthreads();
    if (lane == 63) lds16[wid] = incl;
    __syncthreads();
    double off = incl - run;
    for (int k = 0; k < wid; ++k) off += lds16[k];
    for (int b = b0; b < b1; ++b) {
        out[b] = off;
        off += in[b];
    }
}

// The chain's values inside one unit from its exact entry value s (the value
// before the unit's first term; `first`: the unit's first term starts the chain).
// One term per lane, lanes >= cnt ignored.  While s stays in its binade and no
// term is a rounding tie, the values are s + (prefix of rint(a / u)) u, computed
// for all lanes at once; the first lane where that fails (the sum reaches the
// next binade, a tie, a term < 0 or not finite) takes one plain fp64 add --
// exactly the reference's step -- and the rest restart from there.  Returns the
// lane's value; s becomes the unit's last value.
__device__ inline double chain_unit(double a, int cnt, double &s, bool first) {
    const int lane = threadIdx.x & 63;
    double mine = 0.0;
    int j0 = 0;
    if (first && cnt > 0) {
        s = bcast(a, 0);
        if (lane == 0) mine = s;
        j0 = 1;
    }
    while (j0 < cnt) {
        const bool active = lane >= j0 && lane < cnt;
        if (s == 0.0) {
            // a run of zero terms keeps the chain at 0
            const unsigned long long nz = __ballot(active && a != 0.0);
            const int jn = nz ? (int)__builtin_ctzll(nz) : cnt;
            if (active && lane < jn) mine = s;
            if (jn >= cnt) break;
            s = s + bcast(a, jn);
            if (lane == jn) mine = s;
            j0 = jn + 1;
            continue;
        }
        if (!(s >= 0.0 && s < 0x1p1020)) {                 // outside the regular grid: one step
            s = s + bcast(a, j0);
            if (lane == j0) mine = s;
            ++j0;
            continue;
        }
        const int E = chain_binade(s);
        const double u = unit_ulp(E), top = ldexp(1.0, E + 1);
        const double q = active ? scaled(a, E) : 0.0;
        const bool ok = active && a >= 0.0 && q < 0x1p53;    // false for NaN, inf, negative
        const double fq = ok ? floor(q) : 0.0;
        const long long r = ok ? (long long)rint(q) : 0;
        const long long P = wave_incl_scan_i64(r);
        const double v = s + (double)P * u;
        const bool bad = active && (!ok || q - fq == 0.5 || v >= top);
        const unsigned long long bm = __ballot(bad);
        const int js = bm ? (int)__builtin_ctzll(bm) : cnt;
        if (active && lane < js) mine = v;
        if (js >= cnt) {
            s = bcast(v, cnt - 1);
            break;
        }
        const double sp = (js == j0) ? s : bcast(v, js - 1);
        s = sp + bcast(a, js);
        if (lane == js) mine = s;
        j0 = js + 1;
    }
    return mine;
}

// The binade of the chain at the last translation unit proper (not an identity
// unit) at or before unit k -- the binade of every translation run that ends
// after it, up to the next listed unit: the chain's binade is constant along a run
// of translation and identity units, and a run of identity units alone adds 0
// (then any binade will do: 0 when there is none).
__device__ __forceinline__ int chain_elast(const int32_t *uel, const int32_t *bpe, int64_t k) {
    const int u = uel[k], b = bpe[k / kChainGroup];     // both requested at once
    const int e = u ? u : b;
    return e ? e - 4096 : 0;
}

// Chain value before unit k's first term, for a translation unit; E: the binade
// of the translation run before k (chain_elast(k - 1)).
__device__ __forceinline__ double chain_unit_entry(const ChainView &V, int64_t k, int E) {
    const int64_t g = k / kChainGroup;
    const int o = V.bpc[g] + V.uol[k] - 1;            // the last listed unit before k (unit 0 is listed)
    const int64_t q = V.seql[o];
    const unsigned long long ugk = V.bpd[g] + V.ugl[k], ugq = V.bpd[q / kChainGroup] + V.ugl[q];
    return V.sout[o] + (double)(long long)(ugk - ugq) * unit_ulp(E);
}

// ------------------------------------------------------- numpy sum of w^2 --

// numpy's pairwise_sum leaf (loops_utils.h.src, n <= 128) of the squares of x(0 ..
// len - 1), one thread: n < 8 sequential from 0; else 8 accumulators over the
// full 8-groups, combined ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then
// the rest in order.
template <typename X>
__device__ inline double np_leaf_seq(X x, int len) {
    if (len < 8) {
        double res = 0.0;
        for (int i = 0; i < len; ++i) res += x(i) * x(i);
        return res;
    }
    double r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = x(k) * x(k);
    const int full = len - len % 8;
    for (int i = 8; i < full; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] += x(i + k) * x(i + k);
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (int i = full; i < len; ++i) res += x(i) * x(i);
    return res;
}

// The leaves of a numpy chunk of m elements (m = kNpChunk: 64 leaves of 128;
// else the partial chunk's plan).
__device__ __forceinline__ int np_chunk_leaves(int m, const NpTailPlan *pl) { return m == kNpChunk ? 64 : pl->nl; }
__device__ __forceinline__ int np_leaf_off(int m, const NpTailPlan *pl, int k) { return m == kNpChunk ? 128 * k : pl->off[k]; }
__device__ __forceinline__ int np_leaf_len(int m, const NpTailPlan *pl, int k) { return m == kNpChunk ? 128 : pl->len[k]; }

// The chunk's sum from its leaf values node[0 .. nl) (overwritten): a balanced tree
// in order for a full chunk, the plan's post-order nodes for a partial one.  One thread.
__device__ inline double np_chunk_combine(double *node, int m, const NpTailPlan *pl) {
    if (m == kNpChunk) {
        for (int w = 1; w < 64; w <<= 1)
            for (int k = 0; k < 64; k += 2 * w) node[k] = node[k] + node[k + w];
        return node[0];
    }
    const int nl = pl->nl;
    for (int q = 0; q + 1 < nl; ++q) node[nl + q] = node[pl->a[q]] + node[pl->b[q]];
    return node[2 * nl - 2];
}

// numpy's recursion over n < 8192 elements (n > 128: halves at n/2 rounded down
// to a multiple of 8; leaves of <= 128).
// One wave: numpy's pairwise sum of x[i]^2 over the partial chunk planned by pl.
// The wave sums the leaves 8 lanes per leaf (accumulator k of numpy's 8, 16
// loads in flight), lane 0 runs the plan's adds.  Returns lane 0's value.
__device__ inline double np_pairwise_wave(const double *x, const NpTailPlan *pl) {
    __shared__ double s_node[2 * kNpMaxLeaves];
    const int lane = threadIdx.x & 63;
    const int nl = pl->nl;
    const int grp = lane >> 3, k = lane & 7;
    for (int l0 = 0; l0 < nl; l0 += 8) {
        const int l = l0 + grp;
        const bool in = l < nl;
        const int off = in ? pl->off[l] : 0, len = in ? pl->len[l] : 0;
        const int full = len - len % 8;
        double r = 0.0;
        if (in && len >= 8) {
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = (8 * q + k < full) ? x[off + 8 * q + k] : 0.0;
            r = v[0] * v[0];
#pragma unroll
            for (int q = 1; q < 16; ++q)
                if (8 * q + k < full) r += v[q] * v[q];
        }
        r += __shfl_xor(r, 1, 64);             // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))
        r += __shfl_xor(r, 2, 64);
        r += __shfl_xor(r, 4, 64);
        if (in && k == 0) {
            double res = (len < 8) ? 0.0 : r;
            for (int e = (len < 8) ? 0 : full; e < len; ++e) res += x[off + e] * x[off + e];
            s_node[l] = res;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    double v = 0.0;
    if (lane == 0) {
        for (int q = 0; q + 1 < nl; ++q) s_node[nl + q] = s_node[pl->a[q]] + s_node[pl->b[q]];
        v = s_node[2 * nl - 2];
    }
    return v;
}

}  // namespace fs2
