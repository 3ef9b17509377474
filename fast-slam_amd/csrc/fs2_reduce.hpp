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

// Page of slot j of physical map p.  Slots 4g..4g+3 never straddle a page.
__device__ __forceinline__ char *page_of(char *const *arenas, int j, int32_t p) {
    return arenas[j >> 6] + (int64_t)p * kPageBytes;
}

__device__ __forceinline__ float4 load_mirror(const char *page, int j) {
    return reinterpret_cast<const float4 *>(page)[j & (kPageSlots - 1)];
}

__device__ __forceinline__ Slot load_slot(const char *page, int j) {
    const double2 *q =
        reinterpret_cast<const double2 *>(page + kMirrorBytes + (j & (kPageSlots - 1)) * kSlotBytes);
    const double2 a = q[0], b = q[1], c = q[2];
    return Slot{a.x, a.y, M2{b.x, b.y, c.x, c.y}};
}

// Every slot write keeps the fp32 gate mirror in step with the fp64 slot.
__device__ __forceinline__ void store_slot(char *page, int j, const Slot &s) {
    double2 *q = reinterpret_cast<double2 *>(page + kMirrorBytes + (j & (kPageSlots - 1)) * kSlotBytes);
    q[0] = make_double2(s.mx, s.my);
    q[1] = make_double2(s.P.a00, s.P.a01);
    q[2] = make_double2(s.P.a10, s.P.a11);
    reinterpret_cast<float4 *>(page)[j & (kPageSlots - 1)] = mirror_of(s);
}

// Gate decisions this close to the threshold could depend on ulp-level
// differences upstream (landmark means after EKF); counted, never altered.
__device__ __forceinline__ unsigned ambiguous(double q, double gate2) {
    return fabs(q - gate2) <= 1e-9 * gate2 ? 1u : 0u;
}

}  // namespace fs2
