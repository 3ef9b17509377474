// fs2_reduce.hpp -- wave/block reductions and map-page access shared by the
// update and resample kernels (gfx950, wave64).
#pragma once

#include "fs2_device.hpp"
#include "fs2_kernels.hpp"

namespace fs2 {

// ------------------------------------------------------------ reductions ---

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// (value, index) argmax, lowest index among equal maxima (Python max).
__device__ __forceinline__ void argmax_combine(double &v, int64_t &i, double v2, int64_t i2) {
    if (v2 > v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

__device__ __forceinline__ void wave_argmax(double &v, int64_t &i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double v2 = __shfl_xor(v, o, 64);
        const int64_t i2 = __shfl_xor(i, o, 64);
        argmax_combine(v, i, v2, i2);
    }
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
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// The counters of this workgroup (NV per lane: counters FIRST .. FIRST+NV-1)
// stored (bit k of `assign` set) or added into its column of cpart
// ([kNumCounters][gridDim.x]) and, when wsum != nullptr, its deterministic
// weight sum (block_sum's tree) stored to *wsum: one LDS exchange, one barrier.
template <int NT, int FIRST, int NV>
__device__ void block_counters(const unsigned (&v)[NV], unsigned long long *cpart, unsigned assign, double w,
                               double *wsum) {
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
        unsigned long long *e = cpart + (int64_t)(FIRST + threadIdx.x) * gridDim.x + blockIdx.x;
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

__device__ __forceinline__ uint4 *pt_entry(const MapRef &m, int row, int64_t i) {
    return m.pt + (int64_t)row * m.n + i;
}

// Page of slot j of particle i (read access).
__device__ __forceinline__ char *page_of(const MapRef &m, int j, int64_t i) {
    return page_ptr(m.pool, pt_entry(m, j / kPageSlots, i)->x);
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

__device__ __forceinline__ void store_rec(char *recs, uint32_t r, const Slot &s) {
    double2 *q = reinterpret_cast<double2 *>(recs + (int64_t)r * kRecBytes);
    q[0] = make_double2(s.mx, s.my);
    q[1] = make_double2(s.P.a00, s.P.a01);
    q[2] = make_double2(s.P.a10, s.P.a11);
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
    uint4 *pe = pt_entry(m, row, i);
    const uint32_t e = pe->x;
    if (e & kOwned) return page_ptr(m.pool, e);
    const uint32_t id = take_page(a, m.n, i, t);
    const v4i *src = reinterpret_cast<const v4i *>(page_ptr(m.pool, e));
    v4i *dst = reinterpret_cast<v4i *>(page_ptr(m.pool, id));
    v4i v[kPageBytes / 16];
#pragma unroll
    for (int u = 0; u < kPageBytes / 16; ++u) v[u] = src[u];
#pragma unroll
    for (int u = 0; u < kPageBytes / 16; ++u) dst[u] = v[u];
    pe->x = id | kOwned;       // same content: the summary stays valid
    ++cow;
    return reinterpret_cast<char *>(dst);
}

// A new, owned page for row `row` of particle i (its first slot is being appended).
__device__ __forceinline__ char *fresh_page(const MapRef &m, int row, int64_t i, const PageAlloc &a,
                                            int &t) {
    const uint32_t id = take_page(a, m.n, i, t);
    pt_entry(m, row, i)->x = id | kOwned;      // summary refreshed by the caller
    return page_ptr(m.pool, id);
}

// Every slot write stores the fp64 record r and the slot's mirror (fp32 gate
// shadow + r) in the page.
__device__ __forceinline__ float4 store_slot(const MapRef &m, char *page, int j, const Slot &s, uint32_t r) {
    store_rec(m.recs, r, s);
    float4 mv = mirror_of(s);
    mv.w = __uint_as_float(r);
    reinterpret_cast<float4 *>(page)[j & (kPageSlots - 1)] = mv;
    return mv;
}

// Page summary after slot j (mirror mv) of particle i was written: the first
// slot appended to a fresh page starts a new summary, otherwise the box grows to include mv and s_min
// takes min(s_min, s).  The result covers every slot now in the page (it may
// also cover values since replaced: still conservative).
__device__ __forceinline__ uint4 merge_summary(uint4 d, const float4 &mv) {
    if (!(isfinite(mv.x) && isfinite(mv.y))) return describe_page(d.x, &mv, 0);
    d.y = half_down(fminf(half_lo(d.y), mv.x)) | (half_up(fmaxf(half_hi(d.y), mv.x)) << 16);
    d.z = half_down(fminf(half_lo(d.z), mv.y)) | (half_up(fmaxf(half_hi(d.z), mv.y)) << 16);
    d.w = __float_as_uint(fminf(__uint_as_float(d.w), mv.z));
    return d;
}

__device__ __forceinline__ void note_write(const MapRef &m, int j, int64_t i, const float4 &mv, bool fresh) {
    uint4 *pe = pt_entry(m, j / kPageSlots, i);
    const uint4 d = *pe;
    *pe = fresh ? describe_page(d.x, &mv, 1) : merge_summary(d, mv);
}

// Recompute the summary of page `row` of particle i from its mirrors (map size c).
__device__ __forceinline__ void refresh_summary(const MapRef &m, int row, int64_t i, int c) {
    uint4 *pe = pt_entry(m, row, i);
    const uint32_t e = pe->x;
    const float4 *mir = reinterpret_cast<const float4 *>(page_ptr(m.pool, e));
    *pe = describe_page(e, mir, min(kPageSlots, c - row * kPageSlots));
}

// Gate decisions this close to the threshold could depend on ulp-level
// differences upstream (landmark means after EKF); counted, never altered.
__device__ __forceinline__ unsigned ambiguous(double q, double gate2) {
    return fabs(q - gate2) <= 1e-9 * gate2 ? 1u : 0u;
}

}  // namespace fs2
