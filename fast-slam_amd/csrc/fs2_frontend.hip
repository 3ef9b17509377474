// fs2_frontend.hip -- gfx950 landmark front-end: the reference's
// LandmarkUtils.get_measurements_to_landmarks (utils/landmark_utils.py:21-89),
// i.e. LineFilter -> HoughTransformation.detect_line_intersections
// (algorithms/hough_transformation.py:14-145) -> GeometryUtils.cluster_points
// (utils/geometry_utils.py:26-62, eps 0.5, min_samples 1) -> corner test, for a
// batch of B scans at once (ragged: scan b is points[offs[b], offs[b+1])).
//
// Stages (one HIP launch each, every scan of the batch in the same launch):
//   k_fe_prep    LineFilter + image geometry (min/max of int(100 p))      [B]
//   k_fe_raster  OpenCV's filled radius-2 circle (13-pixel diamond) per point
//                into a per-scan bitmap; first setter of a pixel appends it to
//                the scan's lit-pixel list (the image, deduplicated)        [B]
//   k_fe_vote_peaks  one workgroup per strip of R angles of a scan: rows
//                n0-1 .. n0+R of the accumulator in LDS (16-bit counters),
//                r = cvRound(x cos + y sin) in fp32 like HoughLinesStandard, then
//                local maxima (> left/up, >= right/down, > threshold) [180/R x B]
//   (k_fe_vote + k_fe_peaks: the same through an HBM accumulator, for images
//    whose rows do not fit LDS)
//   k_fe_lines   rank sort (votes desc, index asc) -> (rho, theta)            [B]
//   k_fe_isect   every line pair (i < j) in order: numpy float32 algebra,
//                order-preserving compaction, back to metres               [B]
//   k_fe_cluster DBSCAN(eps, 1) = components of the eps-graph (lock-free
//                union-find, links to the smaller root so a root is its
//                component's first point = sklearn's label order), centres as
//                numpy means, corner test against the filtered scan         [B]
// The (distance, angle) of each corner is computed by the host in fs2_api.hip
// with the C library's powf/pow/atan2, which are what the reference's scalar
// `x ** 2` and math.atan2 call (bit-identical inputs to fs2_iterate).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "fs2_frontend.hpp"

namespace fs2 {

namespace {

constexpr int kFeThreads = 1024;
constexpr int kFeSmall = 256;
constexpr double kFeScale = 100.0;   // hough_transformation.py:11
constexpr int kFePad = 20;           // hough_transformation.py:10

// cv2.circle(radius 2, thickness -1): rows -2..2 of half-widths 0, 1, 2, 1, 0
__constant__ int8_t c_dx[13] = {0, -1, 0, 1, -2, -1, 0, 1, 2, -1, 0, 1, 0};
__constant__ int8_t c_dy[13] = {-2, -1, -1, -1, 0, 0, 0, 0, 0, 1, 1, 1, 2};

__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t n) {
    const int64_t p = 2 * n;
    int64_t k = i % p;
    if (k < 0) k += p;
    return (k < n) ? k : p - 1 - k;
}

// numpy's float32 sin / cos (SIMD Cody-Waite reduction + polynomials, FMA):
// np.cos(np.float32) as the reference's __calculate_intersections evaluates it.
__device__ __forceinline__ float np_sincosf(float x, bool cos_op) {
    const float q = rintf(x * 0x1.45f306p-1f);
    float r = __builtin_fmaf(q, -0x1.921fb0p+00f, x);
    r = __builtin_fmaf(q, -0x1.5110b4p-22f, r);
    r = __builtin_fmaf(q, -0x1.846988p-48f, r);
    const float r2 = r * r;
    float c = __builtin_fmaf(0x1.98e616p-16f, r2, -0x1.6c06dcp-10f);
    c = __builtin_fmaf(c, r2, 0x1.55553cp-05f);
    c = __builtin_fmaf(c, r2, -0x1.000000p-01f);
    c = __builtin_fmaf(c, r2, 1.0f);
    float s = __builtin_fmaf(0x1.7d3bbcp-19f, r2, -0x1.a06bbap-13f);
    s = __builtin_fmaf(s, r2, 0x1.11119ap-07f);
    s = __builtin_fmaf(s, r2, -0x1.555556p-03f);
    s = __builtin_fmaf(s, r2, 0.0f);
    s = __builtin_fmaf(s, r, r);
    const int iq = (int)q + (cos_op ? 1 : 0);
    float v = (iq & 1) == 0 ? s : c;
    if ((iq & 2) == 2) v = -v;
    return v;
}

// Exclusive prefix of `flag` over a 1024-thread block; returns the prefix and
// sets `total`.  wsum: 16 ints of LDS.
__device__ __forceinline__ int block_prefix(int flag, int *wsum, int &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long m = __ballot(flag);
    const int in_wave = __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < kFeThreads / 64; ++w) {
        const int v = wsum[w];
        off += (w < wave) ? v : 0;
        tot += v;
    }
    total = tot;
    return off + in_wave;
}

// i < j pair number t (row-major over i) of K items
__device__ __forceinline__ void pair_of(int64_t t, int K, int &i, int &j) {
    auto S = [K](int64_t r) { return r * (2 * (int64_t)K - r - 1) / 2; };
    const double a = 2.0 * K - 1.0;
    int64_t r = (int64_t)((a - sqrt(fmax(a * a - 8.0 * (double)t, 0.0))) * 0.5);
    r = std::max<int64_t>(0, std::min<int64_t>(r, K - 2));
    while (r > 0 && S(r) > t) --r;
    while (r + 1 <= K - 2 && S(r + 1) <= t) ++r;
    i = (int)r;
    j = (int)(t - S(r) + r + 1);
}

__device__ __forceinline__ int uf_load(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int uf_find(int *par, int x) {
    for (;;) {
        const int p = uf_load(par + x);
        if (p == x) return x;
        x = p;
    }
}

// ------------------------------------------------------------- kernels ---

__global__ __launch_bounds__(kFeSmall) void k_fe_prep(const double2 *pts, const int64_t *offs, const double *taps,
                                                      int radius, double2 *filt, FeGeom *geom) {
    const int b = blockIdx.x;
    const int64_t lo = offs[b], n = offs[b + 1] - lo;
    __shared__ double red[4][kFeSmall];
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    double mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += kFeSmall) {
        // LineFilter.filter (line_filter.py:12-21): correlate1d, mode='reflect'
        double v[2];
        for (int c = 0; c < 2; ++c) {
            auto at = [&](int64_t k) {
                const double2 p = pts[lo + reflect_idx(k, n)];
                return c == 0 ? p.x : p.y;
            };
            double acc = at(i) * taps[radius];
            for (int jj = -radius; jj < 0; ++jj) acc += (at(i + jj) + at(i - jj)) * taps[radius + jj];
            v[c] = acc;
        }
        filt[lo + i] = make_double2(v[0], v[1]);
        const double sx = v[0] * kFeScale, sy = v[1] * kFeScale;
        if (!(fabs(sx) < 1e9 && fabs(sy) < 1e9)) bad = 1;    // NaN / inf / absurd extent
        mnx = fmin(mnx, sx);
        mny = fmin(mny, sy);
        mxx = fmax(mxx, sx);
        mxy = fmax(mxy, sy);
    }
    red[0][threadIdx.x] = mnx;
    red[1][threadIdx.x] = mny;
    red[2][threadIdx.x] = mxx;
    red[3][threadIdx.x] = mxy;
    __syncthreads();
    for (int s = kFeSmall / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            red[0][threadIdx.x] = fmin(red[0][threadIdx.x], red[0][threadIdx.x + s]);
            red[1][threadIdx.x] = fmin(red[1][threadIdx.x], red[1][threadIdx.x + s]);
            red[2][threadIdx.x] = fmax(red[2][threadIdx.x], red[2][threadIdx.x + s]);
            red[3][threadIdx.x] = fmax(red[3][threadIdx.x], red[3][threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    FeGeom g{};
    if (n <= 0) {
        g.status = kFeEmpty;
    } else if (bad) {
        g.status = kFeNonFinite;
    } else {
        // int(np.min(p * 100)) etc. (hough_transformation.py:49-61); trunc toward 0
        const int64_t min_x = (int64_t)red[0][0], min_y = (int64_t)red[1][0];
        const int64_t max_x = (int64_t)red[2][0], max_y = (int64_t)red[3][0];
        const int64_t ox = (min_x < 0 ? -min_x : 0) + kFePad, oy = (min_y < 0 ? -min_y : 0) + kFePad;
        const int64_t W = max_x + ox + kFePad, H = max_y + oy + kFePad;
        const int64_t numrho = 2 * (W + H) + 1;
        if (numrho + 2 > kFeMaxRow || W * H >= (int64_t)1 << 31) {
            g.status = kFeTooLarge;
        } else {
            g.ox = (int32_t)ox;
            g.oy = (int32_t)oy;
            g.W = (int32_t)W;
            g.H = (int32_t)H;
            g.numrho = (int32_t)numrho;
        }
    }
    geom[b] = g;
}

__global__ __launch_bounds__(kFeSmall) void k_fe_raster(const double2 *filt, const int64_t *offs, const FeGeom *geom,
                                                        uint32_t *bitmap, uint32_t *pix, int32_t *npix) {
    const int b = blockIdx.x;
    const FeGeom g = geom[b];
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    if (g.status == 0) {
        const int64_t lo = offs[b], n = offs[b + 1] - lo;
        uint32_t *bm = bitmap + g.bm_off;
        for (int64_t t = threadIdx.x; t < 13 * n; t += kFeSmall) {
            const int64_t k = t / 13;
            const int o = (int)(t - 13 * k);
            const double2 p = filt[lo + k];
            // int(point * 100) + offset (hough_transformation.py:65-68)
            const int x = (int)(int64_t)(p.x * kFeScale) + g.ox + c_dx[o];
            const int y = (int)(int64_t)(p.y * kFeScale) + g.oy + c_dy[o];
            const uint32_t bit = (uint32_t)y * (uint32_t)g.W + (uint32_t)x;
            const uint32_t m = 1u << (bit & 31u);
            const uint32_t old = atomicOr(bm + (bit >> 5), m);
            if (!(old & m)) {
                const int s = atomicAdd(&cnt, 1);
                pix[g.pix_off + s] = (uint32_t)x | ((uint32_t)y << 16);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) npix[b] = cnt;
}

__global__ __launch_bounds__(kFeSmall) void k_fe_vote(const FeGeom *geom, const uint32_t *pix, const int32_t *npix,
                                                      const float *tabs, int32_t *acc) {
    extern __shared__ int32_t row[];
    const int n = blockIdx.x, b = blockIdx.y;
    const FeGeom g = geom[b];
    if (g.status != 0) return;
    const int S = g.numrho + 2;
    for (int k = threadIdx.x; k < S; k += kFeSmall) row[k] = 0;
    __syncthreads();
    const float ts = tabs[n], tc = tabs[kFeAngles + n];
    const int half = (g.numrho - 1) / 2;
    const uint32_t *px = pix + g.pix_off;
    const int np = npix[b];
    for (int q = threadIdx.x; q < np; q += kFeSmall) {
        const uint32_t v = px[q];
        // HoughLinesStandard: r = cvRound(j * tabCos[n] + i * tabSin[n]), fp32, no contraction
        const float a = (float)(int)(v & 0xffffu) * tc;
        const float c = (float)(int)(v >> 16) * ts;
        const float sum = a + c;
        const int r = (int)rintf(sum) + half;
        atomicAdd(&row[r + 1], 1);
    }
    __syncthreads();
    int32_t *A = acc + g.acc_off;
    for (int k = threadIdx.x; k < S; k += kFeSmall) {
        A[(int64_t)(n + 1) * S + k] = row[k];
        if (n == 0) A[k] = 0;
        if (n == kFeAngles - 1) A[(int64_t)(kFeAngles + 1) * S + k] = 0;
    }
}

__global__ __launch_bounds__(kFeSmall) void k_fe_peaks(const FeGeom *geom, const int32_t *acc, int threshold,
                                                       int2 *cand, int32_t *ncand, int cap) {
    const int b = blockIdx.y;
    const FeGeom g = geom[b];
    if (g.status != 0) return;
    const int64_t t = (int64_t)blockIdx.x * kFeSmall + threadIdx.x;
    if (t >= (int64_t)kFeAngles * g.numrho) return;
    const int n = (int)(t / g.numrho), r = (int)(t - (int64_t)n * g.numrho);
    const int S = g.numrho + 2;
    const int base = (n + 1) * S + r + 1;
    const int32_t *A = acc + g.acc_off;
    const int32_t v = A[base];
    if (v > threshold && v > A[base - 1] && v >= A[base + 1] && v > A[base - S] && v >= A[base + S]) {
        const int k = atomicAdd(ncand + b, 1);
        if (k < cap) cand[(int64_t)b * cap + k] = make_int2(v, base);
    }
}

// Vote and local maxima fused: one workgroup per strip of R angles of one scan
// holds rows n0-1 .. n0+R of the accumulator in LDS as packed 16-bit counters
// (a scan's lit pixels < 65536), so the accumulator never goes to HBM.  Rows
// -1 and 180 are OpenCV's zero border rows.  Candidates carry the accumulator
// index of the full (182 x (numrho+2)) array, so ranking is unchanged.
__global__ __launch_bounds__(kFeSmall) void k_fe_vote_peaks(const FeGeom *geom, const uint32_t *pix,
                                                            const int32_t *npix, const float *tabs, int R,
                                                            int threshold, int2 *cand, int32_t *ncand, int cap) {
    extern __shared__ uint32_t rows[];
    const int b = blockIdx.y;
    const FeGeom g = geom[b];
    if (g.status != 0) return;
    const int n0 = blockIdx.x * R;
    if (n0 >= kFeAngles) return;
    const int S = g.numrho + 2;
    const int WS = (S + 1) >> 1;
    const int nrows = R + 2;
    for (int k = threadIdx.x; k < nrows * WS; k += kFeSmall) rows[k] = 0u;
    __syncthreads();
    const int half = (g.numrho - 1) / 2;
    const uint32_t *px = pix + g.pix_off;
    const int np = npix[b];
    const int a_lo = max(n0 - 1, 0), a_hi = min(n0 + R, kFeAngles - 1);
    for (int q = threadIdx.x; q < np; q += kFeSmall) {
        const uint32_t v = px[q];
        const float fx = (float)(int)(v & 0xffffu), fy = (float)(int)(v >> 16);
        for (int n = a_lo; n <= a_hi; ++n) {
            // HoughLinesStandard: r = cvRound(j * tabCos[n] + i * tabSin[n]), fp32, no contraction
            const float a = fx * tabs[kFeAngles + n];
            const float c = fy * tabs[n];
            const float sum = a + c;
            const int col = (int)rintf(sum) + half + 1;
            atomicAdd(&rows[(n - n0 + 1) * WS + (col >> 1)], 1u << ((col & 1) << 4));
        }
    }
    __syncthreads();
    auto at = [&](int k, int col) -> int { return (int)((rows[k * WS + (col >> 1)] >> ((col & 1) << 4)) & 0xffffu); };
    // one packed word (two cells) per step; the neighbour tests run only for the
    // rare cells above the threshold
    const int nend = min(n0 + R, kFeAngles);
    for (int t = threadIdx.x; t < (nend - n0) * WS; t += kFeSmall) {
        const int dn = t / WS, w = t - dn * WS;
        const int k = dn + 1;
        const uint32_t word = rows[k * WS + w];
        if ((int)(word & 0xffffu) <= threshold && (int)(word >> 16) <= threshold) continue;
        for (int h = 0; h < 2; ++h) {
            const int col = 2 * w + h;
            if (col < 1 || col > g.numrho) continue;          // border columns
            const int v = at(k, col);
            if (v > threshold && v > at(k, col - 1) && v >= at(k, col + 1) && v > at(k - 1, col) &&
                v >= at(k + 1, col)) {
                const int slot = atomicAdd(ncand + b, 1);
                if (slot < cap) cand[(int64_t)b * cap + slot] = make_int2(v, (n0 + dn + 1) * S + col);
            }
        }
    }
}

__global__ __launch_bounds__(kFeThreads) void k_fe_lines(const FeGeom *geom, const int2 *cand, const int32_t *ncand,
                                                         int cap, float2 *lines, int32_t *nlines) {
    __shared__ int2 c[kFeMaxLines];   // (votes, accumulator index)
    const int b = blockIdx.x;
    const FeGeom g = geom[b];
    const int K = g.status == 0 ? std::min(ncand[b], cap) : 0;
    for (int k = threadIdx.x; k < K; k += kFeThreads) c[k] = cand[(int64_t)b * cap + k];
    __syncthreads();
    const float theta = (float)(M_PI / 180.0);
    const int S = g.numrho + 2;
    const double scale = 1.0 / S;
    for (int k = threadIdx.x; k < K; k += kFeThreads) {
        const int2 me = c[k];
        int rank = 0;
        for (int q = 0; q < K; ++q) {
            const int2 o = c[q];
            rank += (o.x > me.x || (o.x == me.x && o.y < me.y)) ? 1 : 0;
        }
        const int n = (int)floor(me.y * scale) - 1;
        const int r = me.y - (n + 1) * S - 1;
        const float rho = ((float)r - (float)(g.numrho - 1) * 0.5f) * 1.0f;
        const float th = 0.0f + (float)n * theta;
        lines[(int64_t)b * cap + rank] = make_float2(rho, th);
    }
    if (threadIdx.x == 0) nlines[b] = K;
}

__global__ __launch_bounds__(kFeThreads) void k_fe_isect(const FeGeom *geom, const float2 *lines, const int32_t *nlines,
                                                         int cap, int legacy, const int64_t *isect_off, double2 *isect,
                                                         int32_t *nisect) {
    __shared__ float4 L[kFeMaxLines];     // rho, theta, cos, sin
    __shared__ int wsum[kFeThreads / 64];
    __shared__ int base;
    const int b = blockIdx.x;
    const FeGeom g = geom[b];
    const int K = nlines[b];
    for (int k = threadIdx.x; k < K; k += kFeThreads) {
        const float2 l = lines[(int64_t)b * cap + k];
        L[k] = make_float4(l.x, l.y, np_sincosf(l.y, true), np_sincosf(l.y, false));
    }
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    const int64_t T = (int64_t)K * (K - 1) / 2;
    double2 *out = isect + isect_off[b];
    const float fw = (float)g.W, fh = (float)g.H;
    for (int64_t t0 = 0; t0 < T; t0 += kFeThreads) {
        const int64_t t = t0 + threadIdx.x;
        int flag = 0;
        float x = 0.0f, y = 0.0f;
        if (t < T) {
            int i, j;
            pair_of(t, K, i, j);
            const float4 l1 = L[i], l2 = L[j];
            // hough_transformation.py:94-121 in numpy float32 scalar arithmetic
            float ad = fabsf(l1.y - l2.y);
            const float alt = 3.14159274f - ad;      // np.pi - angle_diff (NEP 50: float32)
            if (alt < ad) ad = alt;
            if (!((double)ad < 0.7853981633974483)) {   // np.deg2rad(45)
                const float p = l1.z * l2.w, q = l2.z * l1.w;
                const float det = p - q;
                if (fabsf(det) > 1e-10f) {
                    const float xn1 = l2.w * l1.x, xn2 = l1.w * l2.x;
                    const float yn1 = l1.z * l2.x, yn2 = l2.z * l1.x;
                    x = (xn1 - xn2) / det;
                    y = (yn1 - yn2) / det;
                    flag = (x >= 0.0f && x < fw && y >= 0.0f && y < fh) ? 1 : 0;
                }
            }
        }
        int total;
        const int pos = block_prefix(flag, wsum, total);
        if (flag) {
            // __convert_back_to_original_space (hough_transformation.py:125-145)
            double ox, oy;
            if (legacy) {
                ox = ((double)x - (double)g.ox) / 100.0;
                oy = ((double)y - (double)g.oy) / 100.0;
            } else {
                ox = (double)((x - (float)g.ox) / 100.0f);
                oy = (double)((y - (float)g.oy) / 100.0f);
            }
            out[base + pos] = make_double2(ox, oy);
        }
        __syncthreads();
        if (threadIdx.x == 0) base += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) nisect[b] = base;
}

__global__ __launch_bounds__(kFeThreads) void k_fe_cluster(const FeGeom *geom, const double2 *filt,
                                                           const int64_t *offs, const double2 *isect,
                                                           const int64_t *isect_off, const int32_t *nisect,
                                                           const int32_t *nlines, double eps2, double corner,
                                                           int legacy, int *par_all, int *lab_all, int cap,
                                                           double2 *centres, double2 *corners, int32_t *counts) {
    __shared__ int wsum[kFeThreads / 64];
    __shared__ int base, cbase;
    const int b = blockIdx.x;
    const int n = nisect[b];
    const double2 *P = isect + isect_off[b];
    int *par = par_all + isect_off[b];
    int *lab = lab_all + isect_off[b];
    for (int i = threadIdx.x; i < n; i += kFeThreads) par[i] = i;
    if (threadIdx.x == 0) {
        base = 0;
        cbase = 0;
    }
    __syncthreads();
    // eps-graph edges (sklearn KDTree: rdist = dx*dx + dy*dy <= eps^2)
    const int64_t T = (int64_t)n * (n - 1) / 2;
    for (int64_t t = threadIdx.x; t < T; t += kFeThreads) {
        int i, j;
        pair_of(t, n, i, j);
        const double dx = P[i].x - P[j].x, dy = P[i].y - P[j].y;
        const double a = dx * dx, c = dy * dy;
        if (a + c <= eps2) {
            for (;;) {
                int ri = uf_find(par, i), rj = uf_find(par, j);
                if (ri == rj) break;
                if (ri > rj) {
                    const int tmp = ri;
                    ri = rj;
                    rj = tmp;
                }
                // link the larger root under the smaller: a root is its component's first point
                if (atomicCAS(par + rj, rj, ri) == rj) break;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kFeThreads) lab[i] = uf_find(par, i);
    __syncthreads();
    // cluster numbers = order of first points; par[c] <- first point of cluster c
    for (int i0 = 0; i0 < n; i0 += kFeThreads) {
        const int i = i0 + threadIdx.x;
        const int root = (i < n && lab[i] == i) ? 1 : 0;
        int total;
        const int pos = block_prefix(root, wsum, total);
        if (root) par[base + pos] = i;
        __syncthreads();
        if (threadIdx.x == 0) base += total;
        __syncthreads();
    }
    const int C = base;
    const int64_t lo = offs[b], np = offs[b + 1] - lo;
    for (int c0 = 0; c0 < C; c0 += kFeThreads) {
        const int c = c0 + threadIdx.x;
        int flag = 0;
        double cx = 0.0, cy = 0.0;
        if (c < C) {
            const int r = par[c];
            // numpy mean(axis=0): index-order sums, / intp count in float64
            double sx = 0.0, sy = 0.0;
            float fx = 0.0f, fy = 0.0f;
            int cnt = 0;
            for (int i = r; i < n; ++i) {
                if (lab[i] != r) continue;
                if (legacy) {
                    sx += P[i].x;
                    sy += P[i].y;
                } else {
                    fx += (float)P[i].x;
                    fy += (float)P[i].y;
                }
                ++cnt;
            }
            if (legacy) {
                cx = sx / (double)cnt;
                cy = sy / (double)cnt;
            } else {
                cx = (double)(float)((double)fx / (double)cnt);
                cy = (double)(float)((double)fy / (double)cnt);
            }
            if (c < cap) centres[(int64_t)b * cap + c] = make_double2(cx, cy);
            // __get_corners (landmark_utils.py:66-89)
            for (int64_t k = 0; k < np; ++k) {
                const double2 s = filt[lo + k];
                const double dx = cx - s.x, dy = cy - s.y;
                const double a = dx * dx, e = dy * dy;
                if (sqrt(a + e) <= corner) {
                    flag = 1;
                    break;
                }
            }
        }
        int total;
        const int pos = block_prefix(flag, wsum, total);
        if (flag && cbase + pos < cap) corners[(int64_t)b * cap + cbase + pos] = make_double2(cx, cy);
        __syncthreads();
        if (threadIdx.x == 0) cbase += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        counts[4 * b + 0] = nlines[b];
        counts[4 * b + 1] = n;
        counts[4 * b + 2] = C;
        counts[4 * b + 3] = cbase;
    }
}

__global__ void k_fe_pack(const double2 *src, const int64_t *src_off, const int32_t *cnt, int B, int cap,
                          double2 *dst) {
    const int b = blockIdx.y;
    const int k = blockIdx.x * kFeSmall + threadIdx.x;
    if (b < B && k < std::min(cnt[b], cap)) dst[(int64_t)b * cap + k] = src[src_off[b] + k];
}

template <typename T>
hipError_t grow(FeBuf &buf, size_t count, T **out) {
    const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    if (buf.bytes < bytes) {
        (void)hipFree(buf.ptr);
        buf.ptr = nullptr;
        buf.bytes = 0;
        const size_t want = std::max(bytes, buf.bytes + buf.bytes / 2);
        hipError_t e = hipMalloc(&buf.ptr, want);
        if (e != hipSuccess) return e;
        buf.bytes = want;
    }
    *out = static_cast<T *>(buf.ptr);
    return hipSuccess;
}

#define FE_TRY(expr)                          \
    do {                                      \
        hipError_t e_ = (expr);               \
        if (e_ != hipSuccess) return e_;      \
    } while (0)

}  // namespace

void fe_trig_table(float *tabs) {
    // OpenCV createTrigTable: float angle advanced by the float step, double sin/cos
    const float theta = (float)(M_PI / 180.0);
    float ang = 0.0f;
    for (int n = 0; n < kFeAngles; ang += theta, ++n) {
        tabs[n] = (float)std::sin((double)ang);
        tabs[kFeAngles + n] = (float)std::cos((double)ang);
    }
}

FeWorkspace::~FeWorkspace() {
    for (FeBuf *b : {&offs, &taps, &tabs, &pts, &filt, &geom, &bitmap, &pix, &npix, &acc, &cand, &ncand, &lines,
                     &nlines, &isect_off, &isect, &nisect, &par, &lab, &centres, &corners, &counts, &pack})
        (void)hipFree(b->ptr);
}

hipError_t frontend_run(FeWorkspace &ws, const FeArgs &a, FeHostOut &o, hipStream_t s) {
    const int B = a.B;
    o.status.assign(B, 0);
    o.counts.assign((size_t)4 * B, 0);
    int64_t *d_offs;
    double *d_taps;
    float *d_tabs;
    FE_TRY(grow(ws.offs, (size_t)B + 1, &d_offs));
    FE_TRY(grow(ws.taps, (size_t)2 * a.radius + 1, &d_taps));
    FE_TRY(grow(ws.tabs, (size_t)2 * kFeAngles, &d_tabs));
    float htabs[2 * kFeAngles];
    fe_trig_table(htabs);
    const int64_t total = a.offs[B];
    FE_TRY(hipMemcpyAsync(d_offs, a.offs, sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice, s));
    FE_TRY(hipMemcpyAsync(d_taps, a.taps, sizeof(double) * (2 * a.radius + 1), hipMemcpyHostToDevice, s));
    FE_TRY(hipMemcpyAsync(d_tabs, htabs, sizeof(htabs), hipMemcpyHostToDevice, s));
    const double2 *d_pts = reinterpret_cast<const double2 *>(a.points);
    if (!a.points_on_device) {
        double2 *p;
        FE_TRY(grow(ws.pts, (size_t)total, &p));
        FE_TRY(hipMemcpyAsync(p, a.points, sizeof(double2) * total, hipMemcpyHostToDevice, s));
        d_pts = p;
    }
    double2 *d_filt;
    FeGeom *d_geom;
    FE_TRY(grow(ws.filt, (size_t)total, &d_filt));
    FE_TRY(grow(ws.geom, (size_t)B, &d_geom));
    hipLaunchKernelGGL(k_fe_prep, dim3(B), dim3(kFeSmall), 0, s, d_pts, d_offs, d_taps, a.radius, d_filt, d_geom);
    std::vector<FeGeom> g(B);
    FE_TRY(hipMemcpyAsync(g.data(), d_geom, sizeof(FeGeom) * B, hipMemcpyDeviceToHost, s));
    FE_TRY(hipStreamSynchronize(s));
    // per-scan regions of the pixel list, bitmap and accumulator
    int64_t pix_n = 0, bm_n = 0, acc_n = 0;
    int max_rho = 0;
    for (int b = 0; b < B; ++b) {
        o.status[b] = g[b].status;
        if (g[b].status) continue;
        g[b].pix_off = pix_n;
        g[b].bm_off = bm_n;
        g[b].acc_off = acc_n;
        pix_n += 13 * (a.offs[b + 1] - a.offs[b]);
        bm_n += ((int64_t)g[b].W * g[b].H + 31) / 32;
        acc_n += (int64_t)(kFeAngles + 2) * (g[b].numrho + 2);
        max_rho = std::max(max_rho, g[b].numrho);
    }
    for (int b = 0; b < B; ++b)
        if (o.status[b]) return hipSuccess;         // caller reports the first bad scan
    FE_TRY(hipMemcpyAsync(d_geom, g.data(), sizeof(FeGeom) * B, hipMemcpyHostToDevice, s));
    uint32_t *d_bm, *d_pix;
    int32_t *d_npix, *d_acc = nullptr, *d_ncand;
    FE_TRY(grow(ws.bitmap, (size_t)bm_n, &d_bm));
    FE_TRY(grow(ws.pix, (size_t)pix_n, &d_pix));
    FE_TRY(grow(ws.npix, (size_t)B, &d_npix));
    FE_TRY(grow(ws.ncand, (size_t)B, &d_ncand));
    FE_TRY(hipMemsetAsync(d_bm, 0, sizeof(uint32_t) * bm_n, s));
    hipLaunchKernelGGL(k_fe_raster, dim3(B), dim3(kFeSmall), 0, s, d_filt, d_offs, d_geom, d_bm, d_pix, d_npix);
    // fused vote + maxima when every scan's rows fit LDS as 16-bit counters,
    // otherwise int32 rows per angle through an HBM accumulator
    int64_t max_pix = 0;
    for (int b = 0; b < B; ++b) max_pix = std::max<int64_t>(max_pix, 13 * (a.offs[b + 1] - a.offs[b]));
    const int ws_words = (max_rho + 2 + 1) / 2;
    const int R = std::min(16, kFeFusedLds / (4 * ws_words) - 2);
    const bool fused = R >= 1 && max_pix < 65536;
    if (fused) {
        FE_TRY(hipFuncSetAttribute((const void *)k_fe_vote_peaks, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   kFeFusedLds));
    } else {
        FE_TRY(grow(ws.acc, (size_t)acc_n, &d_acc));
        FE_TRY(hipFuncSetAttribute((const void *)k_fe_vote, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   sizeof(int32_t) * kFeMaxRow));
        hipLaunchKernelGGL(k_fe_vote, dim3(kFeAngles, B), dim3(kFeSmall), sizeof(int32_t) * (size_t)(max_rho + 2), s,
                           d_geom, d_pix, d_npix, d_tabs, d_acc);
    }
    // local maxima; the candidate buffer grows when a scan overflows it
    int cap = std::max(ws.cand_cap, 64);
    std::vector<int32_t> nc(B);
    int2 *d_cand;
    for (;;) {
        FE_TRY(grow(ws.cand, (size_t)B * cap, &d_cand));
        FE_TRY(hipMemsetAsync(d_ncand, 0, sizeof(int32_t) * B, s));
        if (fused) {
            const unsigned gx = (unsigned)((kFeAngles + R - 1) / R);
            hipLaunchKernelGGL(k_fe_vote_peaks, dim3(gx, B), dim3(kFeSmall), sizeof(uint32_t) * (size_t)(R + 2) * ws_words,
                               s, d_geom, d_pix, d_npix, d_tabs, R, a.threshold, d_cand, d_ncand, cap);
        } else {
            const unsigned gx = (unsigned)(((int64_t)kFeAngles * max_rho + kFeSmall - 1) / kFeSmall);
            hipLaunchKernelGGL(k_fe_peaks, dim3(gx, B), dim3(kFeSmall), 0, s, d_geom, d_acc, a.threshold, d_cand,
                               d_ncand, cap);
        }
        FE_TRY(hipMemcpyAsync(nc.data(), d_ncand, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s));
        FE_TRY(hipStreamSynchronize(s));
        const int mx = B ? *std::max_element(nc.begin(), nc.end()) : 0;
        if (mx > kFeMaxLines) {
            for (int b = 0; b < B; ++b)
                if (nc[b] > kFeMaxLines) o.status[b] = kFeTooManyLines;
            return hipSuccess;
        }
        if (mx <= cap) break;
        cap = std::min(kFeMaxLines, std::max(mx, 2 * cap));
    }
    o.fused = fused;
    ws.cand_cap = cap;
    float2 *d_lines;
    int32_t *d_nlines, *d_nisect, *d_counts, *d_par, *d_lab;
    int64_t *d_ioff;
    double2 *d_isect, *d_cent, *d_corn;
    FE_TRY(grow(ws.lines, (size_t)B * cap, &d_lines));
    FE_TRY(grow(ws.nlines, (size_t)B, &d_nlines));
    hipLaunchKernelGGL(k_fe_lines, dim3(B), dim3(kFeThreads), 0, s, d_geom, d_cand, d_ncand, cap, d_lines, d_nlines);
    std::vector<int64_t> ioff(B + 1, 0);
    for (int b = 0; b < B; ++b) ioff[b + 1] = ioff[b] + (int64_t)nc[b] * (nc[b] - 1) / 2;
    FE_TRY(grow(ws.isect_off, (size_t)B + 1, &d_ioff));
    FE_TRY(grow(ws.isect, (size_t)ioff[B], &d_isect));
    FE_TRY(grow(ws.nisect, (size_t)B, &d_nisect));
    FE_TRY(grow(ws.par, (size_t)ioff[B], &d_par));
    FE_TRY(grow(ws.lab, (size_t)ioff[B], &d_lab));
    const int ocap = std::max(a.cap, 1);
    FE_TRY(grow(ws.centres, (size_t)B * ocap, &d_cent));
    FE_TRY(grow(ws.corners, (size_t)B * ocap, &d_corn));
    FE_TRY(grow(ws.counts, (size_t)4 * B, &d_counts));
    FE_TRY(hipMemcpyAsync(d_ioff, ioff.data(), sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_fe_isect, dim3(B), dim3(kFeThreads), 0, s, d_geom, d_lines, d_nlines, cap, a.legacy, d_ioff,
                       d_isect, d_nisect);
    hipLaunchKernelGGL(k_fe_cluster, dim3(B), dim3(kFeThreads), 0, s, d_geom, d_filt, d_offs, d_isect, d_ioff,
                       d_nisect, d_nlines, a.eps * a.eps, a.corner, a.legacy, d_par, d_lab, ocap, d_cent, d_corn,
                       d_counts);
    FE_TRY(hipGetLastError());
    FE_TRY(hipMemcpyAsync(o.counts.data(), d_counts, sizeof(int32_t) * 4 * B, hipMemcpyDeviceToHost, s));
    if (a.cap > 0) {
        const size_t row = sizeof(double2) * a.cap;
        if (o.lines) {
            const size_t w = sizeof(float2) * std::min(a.cap, cap);
            FE_TRY(hipMemcpy2DAsync(o.lines, sizeof(float2) * a.cap, d_lines, sizeof(float2) * cap, w, B,
                                    hipMemcpyDeviceToHost, s));
        }
        if (o.intersections) {
            double2 *d_pack;
            FE_TRY(grow(ws.pack, (size_t)B * a.cap, &d_pack));
            hipLaunchKernelGGL(k_fe_pack, dim3((a.cap + kFeSmall - 1) / kFeSmall, B), dim3(kFeSmall), 0, s, d_isect,
                               d_ioff, d_nisect, B, a.cap, d_pack);
            FE_TRY(hipMemcpyAsync(o.intersections, d_pack, row * B, hipMemcpyDeviceToHost, s));
        }
        if (o.clusters) FE_TRY(hipMemcpyAsync(o.clusters, d_cent, row * B, hipMemcpyDeviceToHost, s));
        if (o.corners) FE_TRY(hipMemcpyAsync(o.corners, d_corn, row * B, hipMemcpyDeviceToHost, s));
    }
    FE_TRY(hipStreamSynchronize(s));
    return hipGetLastError();
}

}  // namespace fs2
