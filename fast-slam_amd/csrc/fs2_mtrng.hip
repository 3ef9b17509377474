// fs2_mtrng.hip -- numpy's legacy MT19937 stream and polar Gaussian on the device
// (fs2_mtrng.hpp): the drop-in iterate()'s motion draws (fast_slam_2.py:79,81)
// and resample start (:183) bit for bit with np.random, without the host
// generating N normals per scan.
//
//   k_mt_words    one workgroup: the raw word stream, 623 words (2.7 steps of
//                 the recurrence) per barrier, a thread per 227-strided chain,
//                 the last 2048 words in an LDS ring;
//   k_mt_count    one lane per polar attempt (4 words): accepted attempts per
//                 256-attempt block;
//   k_mt_scan     one workgroup: exclusive offsets of the block counts;
//   k_mt_normals  one lane per attempt: its rank among the accepted attempts
//                 gives its two output indices; log in double-double, results
//                 near a rounding midpoint listed for the host (libm log);
//   k_mt_patch    the host's recomputed values into the output.
#include "fs2_kernels.hpp"
#include "fs2_mtrng.hpp"

namespace fs2 {

// A phase makes the 623 words [base, base + 623): thread q < 227 the words
// base + q, base + q + 227 and (q < 169) base + q + 454, each one's x[j - 227]
// being the thread's previous word except the first's (read, like every
// x[j - 624], x[j - 623], from the LDS ring).  Every word read is older than the
// phase (623 = 624 - 1 is the most a phase can make), so one barrier per phase
// orders the ring.  The ring holds 2048 words, mirrored (word i at i mod 2048 and
// i mod 2048 + 2048) so the pair x[j - 624], x[j - 623] never wraps; a phase reads
// [base - 624, base) and writes [base, base + 623), never the same slots.
constexpr int kMtPhase = 2 * kMtLag + (kMtN - 1 - 2 * kMtLag);   // 623
__global__ __launch_bounds__(256) void k_mt_words(uint32_t *R, int64_t begin, int64_t end) {
    __shared__ uint32_t ring[4096];
    const int q = threadIdx.x;
    for (int t = q; t < kMtN; t += 256) {
        const int64_t j = begin - kMtN + t;
        const uint32_t v = R[j];
        ring[j & 2047] = v;
        ring[(j & 2047) + 2048] = v;
    }
    __syncthreads();
    const bool on = q < kMtLag, on2 = q < kMtPhase - 2 * kMtLag;
    for (int64_t base = begin; base < end; base += kMtPhase) {
        const int64_t j0 = base + q, j1 = j0 + kMtLag, j2 = j1 + kMtLag;
        if (on) {
            const uint32_t c0 = ring[(j0 - kMtLag) & 2047];
            const uint32_t *p0 = ring + ((j0 - kMtN) & 2047);
            const uint32_t *p1 = ring + ((j1 - kMtN) & 2047);
            const uint32_t *p2 = ring + ((j2 - kMtN) & 2047);
            const uint32_t a0 = p0[0], b0 = p0[1], a1 = p1[0], b1 = p1[1];
            const uint32_t a2 = p2[0], b2 = p2[1];   // (read by every thread: one round trip)
            const uint32_t v0 = mt_next_word(a0, b0, c0);
            const uint32_t v1 = mt_next_word(a1, b1, v0);
            ring[j0 & 2047] = v0;
            ring[(j0 & 2047) + 2048] = v0;
            ring[j1 & 2047] = v1;
            ring[(j1 & 2047) + 2048] = v1;
            if (j0 < end) R[j0] = v0;
            if (j1 < end) R[j1] = v1;
            if (on2) {
                const uint32_t v2 = mt_next_word(a2, b2, v1);
                ring[j2 & 2047] = v2;
                ring[(j2 & 2047) + 2048] = v2;
                if (j2 < end) R[j2] = v2;
            }
        }
        // the phase's LDS writes complete, then the barrier; the global stores stay
        // in flight (__syncthreads would wait for them too: its workgroup-scope
        // fence covers global memory)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

struct MtParams {
    const uint32_t *R;       // raw stream words x_0 .. (x_0..x_623 = the input key)
    int64_t pos0;            // stream index of the first word to consume
    int64_t A;               // attempts evaluated
    int64_t P;               // accepted attempts needed (pairs)
    int64_t N;               // normals drawn
    int32_t h0;              // the first normal is the cached gauss0
    double gauss0;
    double sigma;            // legacy_normal(0, sigma)
    int64_t first, n_local;  // this rank's slice of the N outputs
    double *out;             // [n_local]
    int32_t *boff;           // [nb] accepted per block -> exclusive offsets
    int32_t nb;
    MtMeta *meta;
    MtAmb *amb;
    int32_t amb_cap;
    const double *tab;       // [2][kMtLogTab] log table (k_mt_table), hi then lo
};

// the log table of mt_log (host and device compute the same bits)
__global__ __launch_bounds__(128) void k_mt_table(double *tab) {
    if (threadIdx.x < kMtLogTab) {
        const DD l = mt_log_tab_entry(threadIdx.x);
        tab[threadIdx.x] = l.hi;
        tab[kMtLogTab + threadIdx.x] = l.lo;
    }
}

__global__ __launch_bounds__(256) void k_mt_count(const MtParams p) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool ok = false;
    if (a < p.A) {
        const uint32_t *w = p.R + p.pos0 + 4 * a;
        ok = mt_attempt(w[0], w[1], w[2], w[3]).ok;
    }
    __shared__ int s_c[4];
    const uint64_t bal = __ballot(ok);
    if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = __popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) p.boff[blockIdx.x] = s_c[0] + s_c[1] + s_c[2] + s_c[3];
}

__global__ __launch_bounds__(1024) void k_mt_scan(const MtParams p) {
    __shared__ int s_w[16];
    __shared__ int64_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int base = 0; base < p.nb; base += 1024) {
        const int b = base + threadIdx.x;
        const int v = b < p.nb ? p.boff[b] : 0;
        // inclusive wave scan
        int x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) s_w[wid] = x;
        __syncthreads();
        int before = 0;
        for (int k = 0; k < wid; ++k) before += s_w[k];
        const int64_t carry = s_carry;
        if (b < p.nb) p.boff[b] = (int32_t)(carry + before + x - v);
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = carry + before + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) p.meta->accepted = s_carry;
}

__global__ __launch_bounds__(256) void k_mt_normals(const MtParams p) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    MtAttempt t{0.0, 0.0, 0.0, false};
    if (a < p.A) {
        const uint32_t *w = p.R + p.pos0 + 4 * a;
        t = mt_attempt(w[0], w[1], w[2], w[3]);
    }
    __shared__ int s_c[4];
    __shared__ double s_thi[kMtLogTab], s_tlo[kMtLogTab];
    if (threadIdx.x < kMtLogTab) {
        s_thi[threadIdx.x] = p.tab[threadIdx.x];
        s_tlo[threadIdx.x] = p.tab[kMtLogTab + threadIdx.x];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t bal = __ballot(t.ok);
    if (lane == 0) s_c[wid] = __popcll(bal);
    __syncthreads();
    int before = 0;
    for (int k = 0; k < wid; ++k) before += s_c[k];
    const int64_t rank = (int64_t)(p.nb > 0 ? p.boff[blockIdx.x] : 0) + before +
                         __popcll(bal & ((1ull << lane) - 1ull));
    if (a == 0 && p.h0) {
        // the cached value of the previous draw comes first
        if (p.first == 0 && p.n_local > 0) p.out[0] = 0.0 + p.sigma * p.gauss0;
    }
    const bool use = t.ok && rank < p.P;
    bool amb = false;
    const double lg = use ? mt_log(t.r2, s_thi, s_tlo, &amb) : 0.0;
    // the block's listed attempts take consecutive entries: one atomic per block
    __shared__ int s_a[4];
    __shared__ int s_abase;
    const uint64_t abal = __ballot(amb);
    if (lane == 0) s_a[wid] = __popcll(abal);
    __syncthreads();
    if (threadIdx.x == 0) {
        const int tot = s_a[0] + s_a[1] + s_a[2] + s_a[3];
        s_abase = tot ? atomicAdd(&p.meta->amb_n, tot) : 0;
    }
    __syncthreads();
    if (amb) {
        int k = s_abase + __popcll(abal & ((1ull << lane) - 1ull));
        for (int w = 0; w < wid; ++w) k += s_a[w];
        if (k < p.amb_cap) p.amb[k] = MtAmb{t.r2, t.x1, t.x2, rank};
    }
    if (!use) return;
    const double f = mt_polar_f(t.r2, lg);
    const double g0 = f * t.x2, g1 = f * t.x1;
    const int64_t o = p.h0 + 2 * rank;
    if (o >= p.first && o < p.first + p.n_local) p.out[o - p.first] = 0.0 + p.sigma * g0;
    if (o + 1 < p.N) {
        if (o + 1 >= p.first && o + 1 < p.first + p.n_local) p.out[o + 1 - p.first] = 0.0 + p.sigma * g1;
    }
    if (rank == p.P - 1) {
        p.meta->last_attempt = a;
        p.meta->has_gauss = (o + 1 < p.N) ? 0 : 1;
        p.meta->gauss = (o + 1 < p.N) ? 0.0 : g1;
    }
}

// numpy's state after the draw: the key block holding the last word consumed
// (pos = words used of it, 624 before the next twist), and the u0 words
__global__ __launch_bounds__(256) void k_mt_final(const uint32_t *R, int64_t pos0, int64_t b_in, int64_t P,
                                                  MtMeta *meta) {
    const int64_t E = P > 0 ? pos0 + 4 * (meta->last_attempt + 1) : pos0;
    const int64_t b1 = (E == pos0) ? b_in : (E - 1) / kMtN, b2 = (E + 1) / kMtN;
    for (int t = threadIdx.x; t < kMtN; t += 256) {
        meta->key_after[t] = R[kMtN * b1 + t];
        meta->key_after_u0[t] = R[kMtN * b2 + t];
    }
    if (threadIdx.x == 0) {
        meta->E = E;
        meta->pos_after = (int32_t)(E - kMtN * b1);
        meta->pos_after_u0 = (int32_t)(E + 2 - kMtN * b2);
        meta->w_u0[0] = R[E];
        meta->w_u0[1] = R[E + 1];
    }
}

__global__ __launch_bounds__(256) void k_mt_patch(double *out, const int64_t *idx, const double *val, int64_t n) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < n) out[idx[k]] = val[k];
}

__global__ __launch_bounds__(256) void k_mt_debug_log(const double *x, int64_t n, double *out, int32_t *amb) {
    __shared__ double s_thi[kMtLogTab], s_tlo[kMtLogTab];
    if (threadIdx.x < kMtLogTab) {
        const DD l = mt_log_tab_entry(threadIdx.x);
        s_thi[threadIdx.x] = l.hi;
        s_tlo[threadIdx.x] = l.lo;
    }
    __syncthreads();
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    bool a = false;
    out[k] = mt_log(x[k], s_thi, s_tlo, &a);
    amb[k] = a ? 1 : 0;
}

hipError_t launch_mt_words(uint32_t *R, int64_t begin, int64_t end, hipStream_t s) {
    if (end <= begin) return hipSuccess;
    hipLaunchKernelGGL(k_mt_words, dim3(1), dim3(256), 0, s, R, begin, end);
    return hipGetLastError();
}

hipError_t launch_mt_draw(const uint32_t *R, int64_t pos0, int64_t b_in, int64_t A, int64_t P, int64_t N, int32_t h0,
                          double gauss0, double sigma, int64_t first, int64_t n_local, double *out,
                          int32_t *boff, MtMeta *meta, MtAmb *amb, int32_t amb_cap, double *tab, int32_t tab_ready,
                          hipStream_t s) {
    MtParams p{};
    p.tab = tab;
    if (!tab_ready) hipLaunchKernelGGL(k_mt_table, dim3(1), dim3(128), 0, s, tab);
    p.R = R;
    p.pos0 = pos0;
    p.A = A;
    p.P = P;
    p.N = N;
    p.h0 = h0;
    p.gauss0 = gauss0;
    p.sigma = sigma;
    p.first = first;
    p.n_local = n_local;
    p.out = out;
    p.boff = boff;
    p.nb = (int32_t)((A + 255) / 256);
    p.meta = meta;
    p.amb = amb;
    p.amb_cap = amb_cap;
    if (p.nb == 0) {
        hipLaunchKernelGGL(k_mt_normals, dim3(1), dim3(256), 0, s, p);   // the cached value alone
    } else {
        hipLaunchKernelGGL(k_mt_count, dim3(p.nb), dim3(256), 0, s, p);
        hipLaunchKernelGGL(k_mt_scan, dim3(1), dim3(1024), 0, s, p);
        hipLaunchKernelGGL(k_mt_normals, dim3(p.nb), dim3(256), 0, s, p);
    }
    hipLaunchKernelGGL(k_mt_final, dim3(1), dim3(256), 0, s, R, pos0, b_in, P, meta);
    return hipGetLastError();
}

hipError_t launch_mt_patch(double *out, const int64_t *idx, const double *val, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mt_patch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, idx, val, n);
    return hipGetLastError();
}

hipError_t launch_mt_debug_log(const double *x, int64_t n, double *out, int32_t *amb, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mt_debug_log, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n, out, amb);
    return hipGetLastError();
}

}  // namespace fs2
