// fs2_geometry.hip -- gfx950 kernels for the stateless helpers of the hot path:
// ICP scan matching (algorithms/icp.py:13-90), LineFilter (line_filter.py:12-21),
// Mahalanobis distance (geometry_utils.py:13-23) and first-match association
// (landmark_utils.py:92-117).
#include "fs2_device.hpp"
#include "fs2_kernels.hpp"

namespace fs2 {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// fp64 wave sum through DPP row shifts and row broadcasts (no LDS traffic):
// lane 63 collects ((row 0 + row 1) + (row 2 + row 3)) of adjacent-first pair
// sums, then every lane reads it.  A fixed tree, so the result is deterministic.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v += dpp_f64<0x111, 0xf>(v);     // row_shr:1
    v += dpp_f64<0x112, 0xf>(v);     // row_shr:2
    v += dpp_f64<0x114, 0xf>(v);     // row_shr:4
    v += dpp_f64<0x118, 0xf>(v);     // row_shr:8  (lane 15 of each row: the row's sum)
    v += dpp_f64<0x142, 0xa>(v);     // row_bcast:15 into rows 1 and 3
    v += dpp_f64<0x143, 0xc>(v);     // row_bcast:31 into rows 2 and 3 (lane 63: the wave's sum)
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
    return __hiloint2double(hi, lo);
}

// ------------------------------------------------------------------- ICP ---
//
// One workgroup per alignment; the target cloud and the moving source cloud
// live in LDS for the whole loop.  Nearest neighbours (icp.py:36, KDTree query)
// through a uniform grid over the target cloud, built once in LDS: each source
// point searches rings of cells outward until the best distance found is
// provably below the distance to any cell not yet searched, so the result is
// the exact fp64 nearest neighbour, lowest index on exact ties, as brute force
// would give.  Centroids / cross-covariance / mean distance by fixed-order
// wave + LDS reductions; rotation by the closed-form 2-D Kabsch angle, which
// equals the reference's SVD + reflection fix (icp.py:76-85).

constexpr int kIcpMaxP = 1024;
#ifndef FS2_ICP_THREADS
#define FS2_ICP_THREADS 1024
#endif
constexpr int kIcpThreads = FS2_ICP_THREADS;
constexpr int kIcpGrid = 32;                 // cells per axis

// Optional per-phase cycle counts of one alignment (build with -DFS2_PHASE_TIMING;
// fs2_debug_icp_phase_times): NN search, centroid sums, covariance sums, update.
#ifdef FS2_PHASE_TIMING
__device__ unsigned long long g_icp_phase[4];
#define ICP_T(k)                                                           \
    do {                                                                   \
        if (threadIdx.x == 0 && blockIdx.x == 0) {                         \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
            if ((k) > 0) g_icp_phase[(k) - 1] += t_ - t_last;              \
            t_last = t_;                                                   \
        }                                                                  \
    } while (0)
hipError_t debug_icp_phase_times(unsigned long long out[4], int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_icp_phase), sizeof(unsigned long long) * 4);
    if (e == hipSuccess && reset) {
        unsigned long long z[4] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_icp_phase), z, sizeof z);
    }
    return e;
}
#else
#define ICP_T(k) do { } while (0)
#endif

struct IcpGrid {
    double x0, y0, hx, hy, ihx, ihy, slack;
};

__device__ __forceinline__ int icp_cell(double v, double v0, double ih) {
    const double c = (v - v0) * ih;
    return !(c >= 0.0) ? 0 : (c >= (double)(kIcpGrid - 1) ? kIcpGrid - 1 : (int)c);   // NaN -> 0
}

// exact nearest target of p: (index, squared distance).  tsort holds the
// targets in cell order (tsort[q] = tgt[cidx[q]]), so a candidate costs one LDS
// load; its index is read only when it improves or ties the best.
__device__ __forceinline__ void icp_nearest(const double2 p, const IcpGrid &g, const int *cstart,
                                            const int16_t *cidx, const double2 *tsort, int &bj,
                                            double &best) {
    const int cx = icp_cell(p.x, g.x0, g.ihx), cy = icp_cell(p.y, g.y0, g.ihy);
    best = INFINITY;
    bj = INT32_MAX;
    for (int r = 0; r < kIcpGrid; ++r) {
        for (int j = max(cy - r, 0); j <= min(cy + r, kIcpGrid - 1); ++j) {
            const bool edge_row = (j == cy - r) || (j == cy + r);
            const int step = (edge_row || r == 0) ? 1 : 2 * r;
            for (int i = cx - r; i <= cx + r; i += step) {
                if (i < 0 || i >= kIcpGrid) continue;
                const int cell = j * kIcpGrid + i;
                for (int q = cstart[cell]; q < cstart[cell + 1]; ++q) {
                    const double2 tp = tsort[q];
                    const double dx = p.x - tp.x, dy = p.y - tp.y;
                    const double d2 = dx * dx + dy * dy;
                    if (d2 <= best) {
                        const int t = cidx[q];
                        if (d2 < best || t < bj) {
                            best = d2;
                            bj = t;
                        }
                    }
                }
            }
        }
        // distance from p to the cells outside the searched block (those that exist)
        double bound = INFINITY;
        if (cx + r < kIcpGrid - 1) bound = fmin(bound, g.x0 + (cx + r + 1) * g.hx - p.x);
        if (cx - r > 0) bound = fmin(bound, p.x - (g.x0 + (cx - r) * g.hx));
        if (cy + r < kIcpGrid - 1) bound = fmin(bound, g.y0 + (cy + r + 1) * g.hy - p.y);
        if (cy - r > 0) bound = fmin(bound, p.y - (g.y0 + (cy - r) * g.hy));
        if (bound == INFINITY) break;                       // every cell searched
        bound -= g.slack;                                   // cell assignment rounding
        if (bound > 0.0 && best < bound * bound * (1.0 - 1e-12)) break;
    }
    if (bj == INT32_MAX) {          // no comparable target (NaN point): brute force keeps index 0
        bj = 0;
        best = INFINITY;
    }
}

template <int NT>
__device__ void block_sum5(double v[5], double *lds) {
#pragma unroll
    for (int q = 0; q < 5; ++q) v[q] = wave_sum(v[q]);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 5; ++q) lds[q * 16 + wid] = v[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < NT / 64; ++k) t += lds[q * 16 + k];
        v[q] = t;
    }
}

__global__ __launch_bounds__(kIcpThreads) void k_icp(int32_t P, const double *src_all,
                                                     const double *tgt_all, int32_t nt,
                                                     int32_t max_iter, double thr, double *R_out,
                                                     double *t_out, int32_t *iters_out) {
    __shared__ double2 s_src[kIcpMaxP];
    __shared__ double2 s_tgt[kIcpMaxP];
    __shared__ double red[5 * 16];
    __shared__ double s_R[4], s_t[2];
    __shared__ int s_stop;
    __shared__ int s_cstart[kIcpGrid * kIcpGrid + 1];
    __shared__ int s_cfill[kIcpGrid * kIcpGrid];
    __shared__ int16_t s_cidx[kIcpMaxP];
    __shared__ double2 s_tsort[kIcpMaxP];   // targets in cell order
    __shared__ IcpGrid s_g;

    const int b = blockIdx.x;
    const int nth = blockDim.x, nw = nth >> 6;   // launch_icp: one thread per source point, whole waves
    const double2 *src = reinterpret_cast<const double2 *>(src_all) + (int64_t)b * P;
    const double2 *tgt = reinterpret_cast<const double2 *>(tgt_all) + (int64_t)b * nt;
    for (int k = threadIdx.x; k < P; k += nth) s_src[k] = src[k];
    for (int k = threadIdx.x; k < nt; k += nth) s_tgt[k] = tgt[k];
    double Rt[4] = {1.0, 0.0, 0.0, 1.0}, tt[2] = {0.0, 0.0};
    double prev = INFINITY;
    int it = 0;
    // ---- grid over the target cloud (fixed for the whole alignment) ----
    for (int k = threadIdx.x; k < kIcpGrid * kIcpGrid; k += nth) s_cfill[k] = 0;
    __syncthreads();
    {
        double v[5] = {INFINITY, INFINITY, INFINITY, INFINITY, 0.0};   // min x, min y, -max x, -max y
        for (int k = threadIdx.x; k < nt; k += nth) {
            const double2 tp = s_tgt[k];
            v[0] = fmin(v[0], tp.x); v[1] = fmin(v[1], tp.y);
            v[2] = fmin(v[2], -tp.x); v[3] = fmin(v[3], -tp.y);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            for (int o = 32; o > 0; o >>= 1) v[q] = fmin(v[q], __shfl_xor(v[q], o, 64));
        const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
        if (lane == 0)
            for (int q = 0; q < 4; ++q) red[q * 16 + wid] = v[q];
        __syncthreads();
        if (threadIdx.x == 0) {
            double m[4];
            for (int q = 0; q < 4; ++q) {
                m[q] = red[q * 16];
                for (int k = 1; k < nw; ++k) m[q] = fmin(m[q], red[q * 16 + k]);
            }
            IcpGrid g;
            const bool ok = isfinite(m[0]) && isfinite(m[1]) && isfinite(m[2]) && isfinite(m[3]);
            g.x0 = ok ? m[0] : 0.0;
            g.y0 = ok ? m[1] : 0.0;
            const double wx = ok ? -m[2] - m[0] : 0.0, wy = ok ? -m[3] - m[1] : 0.0;
            g.hx = wx > 0.0 ? wx / kIcpGrid : 1.0;
            g.hy = wy > 0.0 ? wy / kIcpGrid : 1.0;
            g.ihx = 1.0 / g.hx;
            g.ihy = 1.0 / g.hy;
            // a target may sit a few ulps on the other side of its cell's edge
            g.slack = 1e-9 * (fabs(g.x0) + fabs(g.y0) + wx + wy) + 1e-300;
            if (!ok) g.hx = g.hy = INFINITY;               // non-finite input: one cell
            s_g = g;
        }
        __syncthreads();
    }
    const IcpGrid grid = s_g;
    for (int k = threadIdx.x; k < nt; k += nth) {
        const double2 tp = s_tgt[k];
        atomicAdd(&s_cfill[icp_cell(tp.y, grid.y0, grid.ihy) * kIcpGrid + icp_cell(tp.x, grid.x0, grid.ihx)], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int k = 0; k < kIcpGrid * kIcpGrid; ++k) {
            s_cstart[k] = run;
            run += s_cfill[k];
            s_cfill[k] = s_cstart[k];
        }
        s_cstart[kIcpGrid * kIcpGrid] = run;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nt; k += nth) {
        const double2 tp = s_tgt[k];
        const int cell = icp_cell(tp.y, grid.y0, grid.ihy) * kIcpGrid + icp_cell(tp.x, grid.x0, grid.ihx);
        s_cidx[atomicAdd(&s_cfill[cell], 1)] = (int16_t)k;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < nt; q += nth) s_tsort[q] = s_tgt[s_cidx[q]];
    __syncthreads();
#ifdef FS2_PHASE_TIMING
    unsigned long long t_last = 0;
#endif
    // One source point per thread (the block has ceil(P / 64) waves).  The
    // point's nearest neighbour and its centroid / covariance terms stay in
    // registers; the per-wave partials are added up once, by lanes of wave 0
    // (one lane per sum), not by every thread.
    __shared__ double red2[5 * 16];
    __shared__ double s_cen[5];
    const int k = threadIdx.x, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    while (it < max_iter) {
        ++it;
        ICP_T(0);
        // nearest neighbour (icp.py:36) and the centroid terms
        double v[5] = {0, 0, 0, 0, 0};
        double2 sp = make_double2(0.0, 0.0), tp = make_double2(0.0, 0.0);
        if (k < P) {
            double best;
            int bj;
            sp = s_src[k];
            icp_nearest(sp, grid, s_cstart, s_cidx, s_tsort, bj, best);
            tp = s_tgt[bj];
            v[0] = 0.0 + sp.x; v[1] = 0.0 + sp.y; v[2] = 0.0 + tp.x; v[3] = 0.0 + tp.y; v[4] = 0.0 + sqrt(best);
        }
        ICP_T(1);
#pragma unroll
        for (int q = 0; q < 5; ++q) v[q] = wave_sum_dpp(v[q]);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 5; ++q) red[q * 16 + wid] = v[q];
        }
        __syncthreads();
        if (threadIdx.x < 5) {
            const int q = threadIdx.x;
            double t = 0.0;
            for (int w = 0; w < nw; ++w) t += red[q * 16 + w];
            s_cen[q] = t / P;
        }
        __syncthreads();
        const double cs0 = s_cen[0], cs1 = s_cen[1], ct0 = s_cen[2], ct1 = s_cen[3];
        const double mean = s_cen[4];
        ICP_T(2);
        // cross-covariance of the centred sets (icp.py:73), summed for thread 0
        double h[4] = {0, 0, 0, 0};
        if (k < P) {
            const double a0 = sp.x - cs0, a1 = sp.y - cs1, b0 = tp.x - ct0, b1 = tp.y - ct1;
            h[0] = 0.0 + a0 * b0; h[1] = 0.0 + a0 * b1; h[2] = 0.0 + a1 * b0; h[3] = 0.0 + a1 * b1;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) h[q] = wave_sum_dpp(h[q]);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) red2[q * 16 + wid] = h[q];
        }
        __syncthreads();
        if (wid == 0) {
            double t = 0.0;
            if (lane < 4)
                for (int w = 0; w < nw; ++w) t += red2[lane * 16 + w];
#pragma unroll
            for (int q = 0; q < 4; ++q) h[q] = __shfl(t, q, 64);
        }
        if (threadIdx.x == 0) {
            // rotation angle th = atan2(y, x) of the 2-D Kabsch solution: cos and
            // sin directly as x / r, y / r (the trigonometric form only where r
            // is 0 or not finite)
            const double x = h[0] + h[3], y = h[1] - h[2];
            const double r = sqrt(x * x + y * y);
            double c, s;
            if (r > 0.0 && r < INFINITY) {
                c = x / r;
                s = y / r;
            } else {
                const double th = atan2(y, x);
                c = cos(th);
                s = sin(th);
            }
            const M2 Ri{c, -s, s, c};
            const double t0 = ct0 - fma(Ri.a00, cs0, Ri.a01 * cs1);
            const double t1 = ct1 - fma(Ri.a10, cs0, Ri.a11 * cs1);
            s_R[0] = Ri.a00; s_R[1] = Ri.a01; s_R[2] = Ri.a10; s_R[3] = Ri.a11;
            s_t[0] = t0; s_t[1] = t1;
            s_stop = fabs(prev - mean) < thr ? 1 : 0;
        }
        __syncthreads();
        ICP_T(3);
        // every reader of red / red2 / s_R has passed the barrier above before
        // the next iteration writes them (each thread moves only its own point)
        const double r00 = s_R[0], r01 = s_R[1], r10 = s_R[2], r11 = s_R[3], t0 = s_t[0], t1 = s_t[1];
        if (k < P) s_src[k] = make_double2(fma(sp.y, r01, sp.x * r00) + t0, fma(sp.y, r11, sp.x * r10) + t1);
        const M2 Rn = mm2(M2{r00, r01, r10, r11}, M2{Rt[0], Rt[1], Rt[2], Rt[3]});
        Rt[0] = Rn.a00; Rt[1] = Rn.a01; Rt[2] = Rn.a10; Rt[3] = Rn.a11;
        const double nt0 = fma(r00, tt[0], r01 * tt[1]) + t0;
        const double nt1 = fma(r10, tt[0], r11 * tt[1]) + t1;
        tt[0] = nt0;
        tt[1] = nt1;
        const int stop = s_stop;
        prev = mean;
        ICP_T(4);
        if (stop) break;
    }
    if (threadIdx.x == 0) {
        for (int q = 0; q < 4; ++q) R_out[b * 4 + q] = Rt[q];
        t_out[b * 2] = tt[0];
        t_out[b * 2 + 1] = tt[1];
        if (iters_out) iters_out[b] = it;
    }
}

hipError_t launch_icp(int32_t B, int32_t P, const double *src, const double *tgt, int32_t n_tgt,
                      int32_t max_iter, double thr, double *R, double *t, int32_t *iters,
                      hipStream_t s) {
    if (P > kIcpMaxP || n_tgt > kIcpMaxP) return hipErrorInvalidValue;
    const int nth = std::max(64, (P + 63) / 64 * 64);     // one thread per source point
    hipLaunchKernelGGL(k_icp, dim3(B), dim3(nth), 0, s, P, src, tgt, n_tgt, max_iter, thr,
                       R, t, iters);
    return hipGetLastError();
}

// best_fit_transform alone: Rt = [R00 R01 R10 R11 t0 t1]
__global__ __launch_bounds__(kIcpThreads) void k_best_fit(const double *src_, const double *tgt_,
                                                          int32_t P, double *Rt) {
    __shared__ double red[5 * 16];
    const double2 *src = reinterpret_cast<const double2 *>(src_);
    const double2 *tgt = reinterpret_cast<const double2 *>(tgt_);
    double v[5] = {0, 0, 0, 0, 0};
    for (int k = threadIdx.x; k < P; k += kIcpThreads) {
        v[0] += src[k].x; v[1] += src[k].y; v[2] += tgt[k].x; v[3] += tgt[k].y;
    }
    block_sum5<kIcpThreads>(v, red);
    const double cs0 = v[0] / P, cs1 = v[1] / P, ct0 = v[2] / P, ct1 = v[3] / P;
    double h[5] = {0, 0, 0, 0, 0};
    for (int k = threadIdx.x; k < P; k += kIcpThreads) {
        const double a0 = src[k].x - cs0, a1 = src[k].y - cs1, b0 = tgt[k].x - ct0, b1 = tgt[k].y - ct1;
        h[0] += a0 * b0; h[1] += a0 * b1; h[2] += a1 * b0; h[3] += a1 * b1;
    }
    block_sum5<kIcpThreads>(h, red);
    if (threadIdx.x == 0) {
        const double th = atan2(h[1] - h[2], h[0] + h[3]);
        const double c = cos(th), s = sin(th);
        Rt[0] = c; Rt[1] = -s; Rt[2] = s; Rt[3] = c;
        Rt[4] = ct0 - fma(c, cs0, -s * cs1);
        Rt[5] = ct1 - fma(s, cs0, c * cs1);
    }
}

hipError_t launch_best_fit(const double *src, const double *tgt, int32_t n, double *Rt, hipStream_t s) {
    hipLaunchKernelGGL(k_best_fit, dim3(1), dim3(kIcpThreads), 0, s, src, tgt, n, Rt);
    return hipGetLastError();
}

// ------------------------------------------------------------ LineFilter ---

__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t n) {
    const int64_t p = 2 * n;
    int64_t k = i % p;
    if (k < 0) k += p;
    return (k < n) ? k : p - 1 - k;
}

// scipy correlate1d, symmetric kernel branch, mode='reflect' (ni_filters.c
// order: centre tap first, then (x[i-k] + x[i+k]) * w for k = r..1).
__global__ __launch_bounds__(kBlock) void k_line_filter(const double *in, int32_t n,
                                                        const double *taps, int32_t r,
                                                        double *out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= 2 * (int64_t)n) return;
    const int64_t i = e >> 1;
    const int col = (int)(e & 1);
    double acc = in[reflect_idx(i, n) * 2 + col] * taps[r];
    for (int jj = -r; jj < 0; ++jj)
        acc += (in[reflect_idx(i + jj, n) * 2 + col] + in[reflect_idx(i - jj, n) * 2 + col]) * taps[r + jj];
    out[e] = acc;
}

hipError_t launch_line_filter(const double *in, int32_t n, const double *taps, int32_t r,
                              double *out, hipStream_t s) {
    const unsigned g = (unsigned)((2 * (int64_t)n + kBlock - 1) / kBlock);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(k_line_filter, dim3(g), dim3(kBlock), 0, s, in, n, taps, r, out);
    return hipGetLastError();
}

// ----------------------------------------------------------- mahalanobis ---
__global__ __launch_bounds__(kBlock) void k_mahalanobis(const double *a, const double *b,
                                                        const double *cov, int32_t K, double *out,
                                                        int32_t *singular) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= K) return;
    M2 I;
    if (!inv2(M2{cov[4 * k], cov[4 * k + 1], cov[4 * k + 2], cov[4 * k + 3]}, I)) {
        atomicOr(singular, 1);
        out[k] = NAN;
        return;
    }
    out[k] = sqrt(quad(I, b[2 * k] - a[2 * k], b[2 * k + 1] - a[2 * k + 1]));
}

hipError_t launch_mahalanobis(const double *a, const double *b, const double *cov, int32_t K,
                              double *out, int32_t *singular, hipStream_t s) {
    const unsigned g = (unsigned)((K + kBlock - 1) / kBlock);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mahalanobis, dim3(g), dim3(kBlock), 0, s, a, b, cov, K, out, singular);
    return hipGetLastError();
}

// ------------------------------------------------------------- associate ---
// One wave walks the list 64 landmarks at a time; the first match (or the
// first singular covariance, where the reference raises) in list order wins.
__global__ __launch_bounds__(64) void k_associate(const double *obs, const double *lm, int32_t L,
                                                  double gate2, int32_t *out) {
    const int lane = threadIdx.x;
    const double ox = obs[0], oy = obs[1];
    for (int base = 0; base < L; base += 64) {
        const int j = base + lane;
        bool match = false, sing = false;
        if (j < L) {
            const double *s = lm + (int64_t)j * 6;
            M2 I;
            if (!inv2(M2{s[2], s[3], s[4], s[5]}, I)) {
                sing = true;
            } else {
                const double q = quad(I, ox - s[0], oy - s[1]);
                match = q >= 0.0 && q < gate2;
            }
        }
        const unsigned long long ev = __ballot(match || sing);
        if (ev) {
            const int first = __ffsll((long long)ev) - 1;
            if (lane == first) out[0] = sing ? -2 : j;
            return;
        }
    }
    if (lane == 0) out[0] = -1;
}

hipError_t launch_associate(const double *obs, const double *lm, int32_t L, double gate2,
                            int32_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_associate, dim3(1), dim3(64), 0, s, obs, lm, L, gate2, out);
    return hipGetLastError();
}

}  // namespace fs2
