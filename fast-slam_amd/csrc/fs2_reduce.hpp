// fs2_reduce.hpp -- wave/block reductions and map-page access shared by the
// update and resample kernels (gfx950, wave64).
#pragma once

#include "fs2_device.hpp"
#include "fs2_kernels.hpp"

namespace fs2 {

// Optional stamps of the tail kernels (build with -DFS2_PHASE_TIMING; read with
// fs2_debug_tail_times): workgroup 0, thread 0, s_memrealtime (100 MHz) deltas
// summed per slot; slot base + k - 1 gets the time from stamp k - 1 to stamp k.
#ifdef FS2_PHASE_TIMING
// one copy per translation unit (no relocatable device code); each unit with
// stamps defines its reader with FS2_TAIL_READER, fs2_debug_tail_times adds them
static __device__ unsigned long long g_tail[32];
#define FS2_TAIL_READER(name)                                                                \
    hipError_t name(unsigned long long out[32], int reset) {                                 \
        hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tail), sizeof(unsigned long long) * 32); \
        if (e == hipSuccess && reset) {                                                      \
            unsigned long long z[32] = {};                                                   \
            e = hipMemcpyToSymbol(HIP_SYMBOL(g_tail), z, sizeof z);                          \
        }                                                                                    \
        return e;                                                                            \
    }
#define FS2_TS_DECL unsigned long long ts_last_ = 0
#define FS2_TS(base, k)                                                                      \
    do {                                                                                     \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                           \
            const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                  \
            if ((k) > 0) atomicAdd(&g_tail[(base) + (k) - 1], t_ - ts_last_);               \
            ts_last_ = t_;                                                                   \
        }                                                                                    \
    } while (0)
#else
#define FS2_TS_DECL do { } while (0)
#define FS2_TS(base, k) do { } while (0)
#endif

// ------------------------------------------------------------ reductions ---
//
// Wave scans and reductions on DPP (gfx9 row_shr 1/2/4/8, then row_bcast 15/31):
// six VALU steps with the neighbour's value as an operand modifier, no LDS
// traffic (a __shfl_* is a ds_bpermute through the LDS crossbar; the reductions
// at the end of every update kernel cost ~100 of them per wave).  After the six
// steps lane l holds the inclusive scan of lanes 0..l (Hillis-Steele inside each
// 16-lane row, then the rows' totals carried up) and lane 63 the wave's
// reduction, which readlane broadcasts (the same bits in every lane).  Every
// lane of the wave must be active.  A lane whose source is out of its row
// reads `id` (the operation's identity).

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp32(uint32_t v, uint32_t id) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64(uint64_t v, uint64_t id) {
    return (uint64_t)dpp32<CTRL, ROWS>((uint32_t)v, (uint32_t)id) |
           ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(v >> 32), (uint32_t)(id >> 32)) << 32);
}
template <typename T>
__device__ __forceinline__ uint64_t to_bits(T v) {
    if constexpr (sizeof(T) == 8) return __builtin_bit_cast(uint64_t, v);
    else return (uint64_t)__builtin_bit_cast(uint32_t, v);
}
template <typename T>
__device__ __forceinline__ T from_bits(uint64_t b) {
    if constexpr (sizeof(T) == 8) return __builtin_bit_cast(T, b);
    else return __builtin_bit_cast(T, (uint32_t)b);
}
template <int CTRL, int ROWS, typename T>
__device__ __forceinline__ T dpp_move(T v, T id) {
    if constexpr (sizeof(T) == 8) return from_bits<T>(dpp64<CTRL, ROWS>(to_bits(v), to_bits(id)));
    else return from_bits<T>(dpp32<CTRL, ROWS>((uint32_t)to_bits(v), (uint32_t)to_bits(id)));
}
template <typename T>
__device__ __forceinline__ T lane63(T v) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t b = to_bits(v);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 63);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63);
        return from_bits<T>((uint64_t)lo | ((uint64_t)hi << 32));
    } else {
        return from_bits<T>((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)to_bits(v), 63));
    }
}
// inclusive scan of op over the wave (op associative and commutative)
template <typename T, typename Op>
__device__ __forceinline__ T dpp_scan(T v, T id, Op op) {
    v = op(v, dpp_move<0x111, 0xf>(v, id));     // row_shr:1
    v = op(v, dpp_move<0x112, 0xf>(v, id));     // row_shr:2
    v = op(v, dpp_move<0x114, 0xf>(v, id));     // row_shr:4
    v = op(v, dpp_move<0x118, 0xf>(v, id));     // row_shr:8
    v = op(v, dpp_move<0x142, 0xa>(v, id));     // row_bcast:15 into rows 1, 3
    v = op(v, dpp_move<0x143, 0xc>(v, id));     // row_bcast:31 into rows 2, 3
    return v;
}

__device__ __forceinline__ double wave_sum(double v) {
    return lane63(dpp_scan(v, 0.0, [](double a, double b) { return a + b; }));
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    return lane63(dpp_scan(v, 0ull, [](unsigned long long a, unsigned long long b) { return a + b; }));
}

__device__ __forceinline__ int wave_max_i(int v) {
    return lane63(dpp_scan(v, INT_MIN, [](int a, int b) { return max(a, b); }));
}

// (value, index) argmax, lowest index among equal maxima (Python max).
__device__ __forceinline__ void argmax_combine(double &v, int64_t &i, double v2, int64_t i2) {
    if (v2 > v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

template <int CTRL, int ROWS>
__device__ __forceinline__ void argmax_step(double &v, int64_t &i) {
    const double v2 = dpp_move<CTRL, ROWS, double>(v, -(double)INFINITY);
    const int64_t i2 = dpp_move<CTRL, ROWS, int64_t>(i, (int64_t)INT64_MAX);
    argmax_combine(v, i, v2, i2);
}

__device__ __forceinline__ void wave_argmax(double &v, int64_t &i) {
    argmax_step<0x111, 0xf>(v, i);
    argmax_step<0x112, 0xf>(v, i);
    argmax_step<0x114, 0xf>(v, i);
    argmax_step<0x118, 0xf>(v, i);
    argmax_step<0x142, 0xa>(v, i);
    argmax_step<0x143, 0xc>(v, i);
    v = lane63(v);
    i = lane63(i);
}

// Deterministic block sum (fixed tree), result valid in every thread.
template <int NT>
__device__ double block_sum(double v, double *lds) {
    v = wave_sum(v);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) t += lds[k];
    return t;
}

template <int NT>
__device__ unsigned long long block_sum_u64(unsigned long long v, unsigned long long *lds) {
    v = wave_sum_u64(v);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    unsigned long long t = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) t += lds[k];
    return t;
}

template <int NT>
__device__ void block_argmax(double &v, int64_t &i, double *ldv, int64_t *ldi) {
    wave_argmax(v, i);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) {
        ldv[wid] = v;
        ldi[wid] = i;
    }
    __syncthreads();
    v = ldv[0];
    i = ldi[0];
#pragma unroll
    for (int k = 1; k < NT / 64; ++k) argmax_combine(v, i, ldv[k], ldi[k]);
}

__device__ __forceinline__ unsigned wave_sum_u32(unsigned v) {
    return lane63(dpp_scan(v, 0u, [](unsigned a, unsigned b) { return a + b; }));
}

// The counters of this workgroup (NV per lane: counters FIRST .. FIRST+NV-1)
// stored (bit k of `assign` set) or added into its column of cpart
// ([kNumCounters][nb], column b) and, when wsum != nullptr, its deterministic
// weight sum (block_sum's tree) stored to *wsum: one LDS exchange, one barrier.
template <int NT, int FIRST, int NV>
__device__ void block_counters(const unsigned (&v)[NV], unsigned long long *cpart, int64_t nb, int64_t b,
                               unsigned assign, double w, double *wsum) {
    __shared__ unsigned s_c[NT / 64][NV];
    __shared__ double s_w[NT / 64];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned r[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) r[k] = wave_sum_u32(v[k]);
    const double ws = wave_sum(w);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) s_c[wid][k] = r[k];
        s_w[wid] = ws;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        unsigned long long t = 0;
#pragma unroll
        for (int q = 0; q < NT / 64; ++q) t += s_c[q][threadIdx.x];
        unsigned long long *e = cpart + (int64_t)(FIRST + threadIdx.x) * nb + b;
        if ((assign >> (FIRST + threadIdx.x)) & 1u) *e = t;
        else if (t) *e += t;
    }
    if (wsum && threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < NT / 64; ++q) t += s_w[q];
        *wsum = t;
    }
}

// DevStats field of update counter k (fs2_kernels.hpp kC*).
__device__ __forceinline__ unsigned long long *counter_field(DevStats *st, int k) {
    switch (k) {
        case kCWords: return &st->words;
        case kCGroups: return &st->groups;
        case kCVisited: return &st->visited;
        case kCCandidates: return &st->candidates;
        case kCWritten: return &st->written;
        case kCAmbiguous: return &st->ambiguous;
        case kCAppends: return &st->appends;
        case kCHits: return &st->hits;
        case kCCow: return &st->cow_pages;
        case kCOpened: return &st->opened;
        case kCRefVisits: return &st->ref_visits;
        default: return &st->new_pages;
    }
}

// The update pass's block counters (cpart[counter][nb]) folded into the scan
// statistics by kFoldBlocks 1024-thread workgroups, workgroup cb over a slice of
// the columns (atomics into DevStats: integer sums, order-free).
constexpr int kFoldBlocks = 8;
__device__ inline void fold_counters(const unsigned long long *cpart, int32_t nb, DevStats *stats, int cb,
                                     unsigned long long (*s_c)[kNumCounters]) {
    const int per = (nb + kFoldBlocks - 1) / kFoldBlocks;
    const int b0 = cb * per, b1 = min(nb, b0 + per);
    // every counter column of the slice at once: independent loads, one LDS exchange
    unsigned long long v[kNumCounters] = {};
    for (int b = b0 + threadIdx.x; b < b1; b += 1024) {
#pragma unroll
        for (int k = 0; k < kNumCounters; ++k) v[k] += cpart[(int64_t)k * nb + b];
    }
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kNumCounters; ++k) {
        v[k] = wave_sum_u64(v[k]);
        if (lane == 0) s_c[wid][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < kNumCounters) {
        const int k = threadIdx.x;
        unsigned long long t = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) t += s_c[q][k];
        if (k == kCSingular) {
            if (t) atomicOr(&stats->error_flags, 1);
        } else if (t) {
            atomicAdd(counter_field(stats, k), t);
        }
    }
}

template <int NT>
__device__ int block_max_i(int v, int *lds) {
    v = wave_max_i(v);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    int t = lds[0];
#pragma unroll
    for (int k = 1; k < NT / 64; ++k) t = max(t, lds[k]);
    return t;
}

// ------------------------------------------------------------- map access ---

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ char *page_ptr(char *pool, uint32_t e) {
    return pool + (int64_t)(e & kIdMask) * kPageBytes;
}

__device__ __forceinline__ Desc *pt_entry(const MapRef &m, int row, int64_t i) {
    return m.pt + (int64_t)row * m.n + i;
}

// Page of slot j of particle i (read access).
__device__ __forceinline__ char *page_of(const MapRef &m, int j, int64_t i) {
    return page_ptr(m.pool, *pt_entry(m, j / kPageSlots, i));
}

// Cold readers in page_refs mode (fs2_kernels.hpp PeerMaps): the page a
// descriptor names on whichever rank holds it, and that rank's record pool (the
// records a page's mirrors name live with the page).
__device__ __forceinline__ const char *page_ptr_any(const MapRef &m, uint32_t e) {
    const uint32_t t = m.peers ? ref_tag(e) : 0u;
    return t ? m.peers->pool[t - 1] + (int64_t)ref_id(e) * kPageBytes : page_ptr(m.pool, e);
}
__device__ __forceinline__ const char *recs_of(const MapRef &m, uint32_t e) {
    const uint32_t t = m.peers ? ref_tag(e) : 0u;
    return t ? m.peers->recs[t - 1] : m.recs;
}

__device__ __forceinline__ float4 load_mirror(const char *page, int j) {
    return reinterpret_cast<const float4 *>(page)[j & (kPageSlots - 1)];
}

__device__ __forceinline__ uint32_t mirror_rec(const float4 &m) { return __float_as_uint(m.w); }

// fp64 record r (x, y, P00, P01, P10, P11).
__device__ __forceinline__ Slot load_rec(const char *recs, uint32_t r) {
    const double2 *q = reinterpret_cast<const double2 *>(recs + (int64_t)r * kRecBytes);
    const double2 a = q[0], b = q[1], c = q[2];
    return Slot{a.x, a.y, M2{b.x, b.y, c.x, c.y}};
}

// Record stores are non-temporal: written once per kernel, read in a later scan
// (k_update -5 %).
__device__ __forceinline__ void store_rec(char *recs, uint32_t r, const Slot &s) {
    typedef double v2d __attribute__((ext_vector_type(2)));
    v2d *qv = reinterpret_cast<v2d *>(recs + (int64_t)r * kRecBytes);
    __builtin_nontemporal_store((v2d){s.mx, s.my}, qv);
    __builtin_nontemporal_store((v2d){s.P.a00, s.P.a01}, qv + 1);
    __builtin_nontemporal_store((v2d){s.P.a10, s.P.a11}, qv + 2);
}

// Slot j of a page: its mirror names the record.
__device__ __forceinline__ Slot load_slot(const MapRef &m, const char *page, int j) {
    return load_rec(m.recs, mirror_rec(load_mirror(page, j)));
}

// Next reserved free page / record of lane i (t counts the lane's allocations).
__device__ __forceinline__ uint32_t take_page(const PageAlloc &a, int64_t n, int64_t i, int &t) {
    const uint32_t id = a.freel[a.base + (int64_t)t * n + i];
    ++t;
    return id;
}

__device__ __forceinline__ uint32_t take_rec(const PageAlloc &a, int64_t n, int64_t i, int &t) {
    const uint32_t id = a.rfreel[a.rbase + (int64_t)t * n + i];
    ++t;
    return id;
}

// Page of row `row` of particle i that this lane may write: its own page, or a
// private copy of a shared one (copy-on-write: 128 B; the page table is updated).
__device__ __forceinline__ char *writable_page(const MapRef &m, int row, int64_t i,
                                               const PageAlloc &a, int &t, unsigned &cow) {
    Desc *pe = pt_entry(m, row, i);
    const uint32_t e = *pe;
    if (e & kOwned) return page_ptr(m.pool, e);
    const uint32_t id = take_page(a, m.n, i, t);
    const v4i *src = reinterpret_cast<const v4i *>(page_ptr(m.pool, e));
    v4i *dst = reinterpret_cast<v4i *>(page_ptr(m.pool, id));
    v4i v[kPageBytes / 16];
#pragma unroll
    for (int u = 0; u < kPageBytes / 16; ++u) v[u] = src[u];
#pragma unroll
    for (int u = 0; u < kPageBytes / 16; ++u) dst[u] = v[u];
    *pe = id | kOwned;         // same content: the row box stays valid
    ++cow;
    return reinterpret_cast<char *>(dst);
}

// A new, owned page for row `row` of particle i (its first slot is being appended).
__device__ __forceinline__ char *fresh_page(const MapRef &m, int row, int64_t i, const PageAlloc &a,
                                            int &t) {
    const uint32_t id = take_page(a, m.n, i, t);
    *pt_entry(m, row, i) = id | kOwned;        // (the caller grows the row box)
    return page_ptr(m.pool, id);
}

// Every slot write stores the fp64 record r and the slot's mirror (fp32 gate
// shadow, slot index, r) at position pos of the page.
__device__ __forceinline__ float4 store_slot(const MapRef &m, char *page, int pos, const Slot &s, uint32_t r,
                                             int slot) {
    store_rec(m.recs, r, s);
    float4 mv = with_slot(mirror_of(s), slot);
    mv.w = __uint_as_float(r);
    reinterpret_cast<float4 *>(page)[pos & (kPageSlots - 1)] = mv;
    return mv;
}

// ---- page summaries (fs2_kernels.hpp) ----

// Grid bound k: org + k cell, exact in fp64 (org and cell are fp32, |k| < 2^8, so
// the product and the sum need < 50 bits).  The cell need not be a power of two
// (round 6: a cell fitted to the maps' extent, not rounded up to one, halves the
// boxes' quantisation slack); every code is checked against these exact bounds.
__device__ __forceinline__ double sum_grid(const SumFrame &f, double k) { return (double)f.org + k * (double)f.cell; }
// Code of the largest grid bound <= v (0: unbounded) / of the smallest >= v (255).
__device__ __forceinline__ uint32_t sum_lo(const SumFrame &f, float v) {
    // (v - org) / cell through the rounded reciprocal: off by < 2^-16 cells, so k is
    // at most one code off -- a step too low is merely conservative, a step too
    // high is undone against the exact bound below (at most once)
    double k = floor(((double)v - (double)f.org) * (double)f.icell);
    if (!(k >= 0.0)) return 0u;          // (also NaN)
    k = fmin(k, 254.0);
    while (k >= 0.0 && sum_grid(f, k) > (double)v) k -= 1.0;
    return k >= 0.0 ? (uint32_t)k + 1u : 0u;
}
__device__ __forceinline__ uint32_t sum_hi(const SumFrame &f, float v) {
    double k = ceil(((double)v - (double)f.org) * (double)f.icell);
    if (!(k <= 254.0)) return 255u;      // (also NaN)
    k = fmax(k, 0.0);
    while (k <= 254.0 && sum_grid(f, k) < (double)v) k += 1.0;
    return k <= 254.0 ? (uint32_t)k : 255u;
}
// the bounds as fp32, rounded outwards (the fp32 page test stays conservative)
__device__ __forceinline__ float sum_lo_val(const SumFrame &f, uint32_t c) {
    return c == 0u ? -INFINITY : __double2float_rd(sum_grid(f, (double)(c - 1u)));
}
__device__ __forceinline__ float sum_hi_val(const SumFrame &f, uint32_t c) {
    return c == 255u ? INFINITY : __double2float_ru(sum_grid(f, (double)c));
}

// Box of the first nvalid mirrors of a page on the grid, or the unbounded box
// when a mirror is not finite or has s = 0 (never reject).
__device__ __forceinline__ uint32_t page_box(const float4 *mir, int nvalid, const SumFrame &f) {
    float xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY, smin = INFINITY;
    bool finite = nvalid > 0;
    for (int u = 0; u < nvalid; ++u) {
        const float4 m = mir[u];
        finite &= isfinite(m.x) && isfinite(m.y);
        xmin = fminf(xmin, m.x);
        xmax = fmaxf(xmax, m.x);
        ymin = fminf(ymin, m.y);
        ymax = fmaxf(ymax, m.y);
        smin = fminf(smin, mirror_s(m));
    }
    if (!finite || !(smin > 0.0f)) return kSumOpen;
    return sum_lo(f, xmin) | (sum_hi(f, xmax) << 8) | (sum_lo(f, ymin) << 16) | (sum_hi(f, ymax) << 24);
}

// Box of one written mirror mv (a box a row's box grows by: it may also cover
// values since replaced, still conservative); unbounded when mv is not finite or
// has s = 0.
__device__ __forceinline__ uint32_t point_box(const float4 &mv, const SumFrame &f) {
    if (!(isfinite(mv.x) && isfinite(mv.y)) || !(mirror_s(mv) > 0.0f)) return kSumOpen;
    return sum_lo(f, mv.x) | (sum_hi(f, mv.x) << 8) | (sum_lo(f, mv.y) << 16) | (sum_hi(f, mv.y) << 24);
}

// ---- workgroup row boxes (fs2_kernels.hpp, MapRef::bbox) ----
// A box's bytes (x lo, x hi, y lo, y hi) as two packed 16-bit pairs: lows
// (x lo | y lo << 16, union = min) and highs (x hi | y hi << 16, union = max),
// so a union is one v_pk_min_u16 and one v_pk_max_u16.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kBoxHalf = 0x00ff00ffu;

__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t box_union(uint32_t a, uint32_t b) {
    return pk_min_u16(a & kBoxHalf, b & kBoxHalf) | (pk_max_u16((a >> 8) & kBoxHalf, (b >> 8) & kBoxHalf) << 8);
}

template <int CTRL, int ROWS>
__device__ __forceinline__ void box_dpp_step(uint32_t &lo, uint32_t &hi) {
    lo = pk_min_u16(lo, (uint32_t)__builtin_amdgcn_update_dpp((int)kBoxHalf, (int)lo, CTRL, ROWS, 0xf, false));
    hi = pk_max_u16(hi, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, ROWS, 0xf, false));
}

// Union of the 64 lanes' boxes (every lane of the wave active), in every lane:
// row_shr 1/2/4/8 leave each 16-lane row's union in its lane 15, row_bcast 15/31
// carry them up, lane 63 holds the wave's (the ICP's DPP pattern, fs2_geometry.hip).
__device__ __forceinline__ uint32_t wave_box_union(uint32_t b) {
    uint32_t lo = b & kBoxHalf, hi = (b >> 8) & kBoxHalf;
    box_dpp_step<0x111, 0xf>(lo, hi);
    box_dpp_step<0x112, 0xf>(lo, hi);
    box_dpp_step<0x114, 0xf>(lo, hi);
    box_dpp_step<0x118, 0xf>(lo, hi);
    box_dpp_step<0x142, 0xa>(lo, hi);
    box_dpp_step<0x143, 0xc>(lo, hi);
    lo = (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
    hi = (uint32_t)__builtin_amdgcn_readlane((int)hi, 63);
    return lo | (hi << 8);
}

// A workgroup's row boxes in LDS as the two packed halves of box_union (lows:
// x lo | y lo << 16, highs: x hi | y hi << 16): 2 KB for 256 rows.  A merge is a
// compare-and-swap of the packed min / max, only when the row box grows (rare).
struct BoxLds {
    uint32_t lo[kBBoxRows], hi[kBBoxRows];
};
__device__ __forceinline__ void lds_box_set(BoxLds &s, int r, uint32_t b) {
    s.lo[r] = b & kBoxHalf;
    s.hi[r] = (b >> 8) & kBoxHalf;
}
__device__ __forceinline__ uint32_t lds_box_get(const BoxLds &s, int r) { return s.lo[r] | (s.hi[r] << 8); }
// grow row r's box to hold b
__device__ __forceinline__ void lds_box_merge(BoxLds &s, int r, uint32_t b) {
    const uint32_t blo = b & kBoxHalf, bhi = (b >> 8) & kBoxHalf;
    uint32_t lo = s.lo[r], hi = s.hi[r];
    for (uint32_t want = pk_min_u16(lo, blo); want != lo; want = pk_min_u16(lo, blo)) {
        const uint32_t prev = atomicCAS(&s.lo[r], lo, want);
        if (prev == lo) break;
        lo = prev;
    }
    for (uint32_t want = pk_max_u16(hi, bhi); want != hi; want = pk_max_u16(hi, bhi)) {
        const uint32_t prev = atomicCAS(&s.hi[r], hi, want);
        if (prev == hi) break;
        hi = prev;
    }
}

// Measurements whose band box `s` (page summary or row box) does not lie outside
// (bc: band_codes thresholds of each measurement, gate_band).
template <int MAXM>
__device__ __forceinline__ unsigned box_open_mask(uint32_t s, const uint32_t (&bc)[MAXM], int m) {
    const uint32_t xl = s & 0xffu, xh = (s >> 8) & 0xffu, yl = (s >> 16) & 0xffu, yh = s >> 24;
    unsigned om = 0u;
#pragma unroll
    for (int k = 0; k < MAXM; ++k)
        if (k < m && xl <= (bc[k] & 0xffu) && xh >= ((bc[k] >> 8) & 0xffu) && yl <= ((bc[k] >> 16) & 0xffu) &&
            yh >= (bc[k] >> 24))
            om |= 1u << k;
    return om;
}

// True when no slot of the page can pass the gate for the observed point: the
// distance to the box is <= |fx - x_lm| for every slot, the margins use the
// box's largest |x|, and slb <= s of every slot (a slot with s = 0 opened the
// box), and every fp32 operation below is monotone, so the value compared is
// <= gate_reject_fast's value for each slot.
__device__ __forceinline__ bool page_reject(uint32_t sum, const SumFrame &f, float slb, float fx, float fy,
                                            float fe, float gate2f) {
    const float xmin = sum_lo_val(f, sum & 0xffu), xmax = sum_hi_val(f, (sum >> 8) & 0xffu);
    const float ymin = sum_lo_val(f, (sum >> 16) & 0xffu), ymax = sum_hi_val(f, sum >> 24);
    const float Dx = fmaxf(fmaxf(xmin - fx, fx - xmax), 0.0f);
    const float Dy = fmaxf(fmaxf(ymin - fy, fy - ymax), 0.0f);
    const float Cx = fmaxf(fabsf(xmin), fabsf(xmax)) * 2.3841858e-7f;
    const float Cy = fmaxf(fabsf(ymin), fabsf(ymax)) * 2.3841858e-7f;
    const float lx = fmaxf(fmaf(Dx, 0.99999976f, -(fe + Cx)), 0.0f);
    const float ly = fmaxf(fmaf(Dy, 0.99999976f, -(fe + Cy)), 0.0f);
    return slb * fmaf(lx, lx, ly * ly) > gate2f;
}

// ---- measurement bands: the cheap pre-tests of the candidate stream ----
//
// For measurement (fx, fy, fe) every slot with mirror s >= slb > 0 and finite
// fp32 coordinates whose true distance to fx in x alone is D >= Rx is rejected
// by gate_reject_fast, whatever its y:
//   |fl(fx - x)| >= D (1 - 2^-24),  fl(fe + cx) <= (fe + (|fx| + D) 2^-22)(1 + 2^-24),
//   so lx >= D (1 - 6e-7) - (fe + 2^-22 |fx|)(1 + 1e-7) >= L (1 + 1.9e-5)
// with Rx = (L (1 + 1e-5) + fe (1 + 1e-5) + 1e-6 |fx|)(1 + 1e-5), L = sqrt(gate2f / slb);
// then s * fma(lx, lx, ly^2) >= slb lx^2 (1 - 2^-24)^2 > gate2f.  Likewise in y.
// A page summary box lying entirely beyond fx + Rx or fx - Rx holds only such
// slots (a bounded box has finite mirrors with s > 0; kSumOpen is never outside),
// so the page is rejected for that measurement from its 8-bit codes alone.
// Every margin only widens the band, so no slot the slot test keeps is dropped.
struct Band {
    uint32_t cx, cy;   // (a | b << 8): box outside iff low code > a or high code < b
};

__device__ __forceinline__ Band band_none() { return Band{0xffu, 0xffu}; }

// code thresholds of the band [f - R, f + R] on the summary grid: a box with
// lo(xl) >= f + R (xl >= A) or hi(xh) <= f - R (xh <= B) is outside
__device__ inline uint32_t band_codes(double f, double R, const SumFrame &fr) {
    const double cell = fr.cell, org = fr.org;
    if (!(isfinite(R) && isfinite(f) && cell > 0.0)) return 0xffu;   // never outside
    const double ta = (f + R - org) / cell + 1.0 + 1e-6;   // lo(c) = org + (c - 1) cell >= f + R
    const double tb = (f - R - org) / cell - 1e-6;         // hi(c) = org + c cell <= f - R
    const double A = fmin(fmax(ceil(ta), 1.0), 256.0);     // 256: never (codes <= 255)
    const double B = fmin(fmax(floor(tb), -1.0), 254.0);   // -1: never; 255 is unbounded
    return (uint32_t)(A - 1.0) | ((uint32_t)(B + 1.0) << 8);
}

__device__ inline Band gate_band(float fx, float fy, float fe, float slb, float gate2f, const SumFrame &fr) {
    const double L = sqrt((double)gate2f / (double)slb);
    const double base = L * (1.0 + 1e-5) + (double)fe * (1.0 + 1e-5);
    const double Rx = (base + fabs((double)fx) * 1e-6) * (1.0 + 1e-5);
    const double Ry = (base + fabs((double)fy) * 1e-6) * (1.0 + 1e-5);
    Band b;
    b.cx = band_codes(fx, Rx, fr);
    b.cy = band_codes(fy, Ry, fr);
    return b;
}


// slb lowered to the smallest positive s the wave's lanes pass (+inf: none); at
// most one atomic per wave, and only when it lowers the bound.  Call with the
// whole wave converged.
__device__ __forceinline__ void lower_slb(float *slb, float s) {
    float v = (s > 0.0f) ? s : INFINITY;
    v = lane63(dpp_scan(v, INFINITY, [](float a, float b) { return fminf(a, b); }));
    if ((threadIdx.x & 63) == 0 && v < *slb) atomicMin(reinterpret_cast<unsigned *>(slb), __float_as_uint(v));
}

// Gate decisions this close to the threshold could depend on ulp-level
// differences upstream (landmark means after EKF); counted, never altered.
__device__ __forceinline__ unsigned ambiguous(double q, double gate2) {
    return fabs(q - gate2) <= 1e-9 * gate2 ? 1u : 0u;
}

}  // namespace fs2
