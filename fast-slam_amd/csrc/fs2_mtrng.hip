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
#include <algorithm>
#include <vector>

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
// (init: the 624 words before begin)
__device__ __forceinline__ void mt_words_body(uint32_t *R, int64_t begin, int64_t end, const uint32_t *init) {
    __shared__ uint32_t ring[4096];
    const int q = threadIdx.x;
    for (int t = q; t < kMtN; t += 256) {
        const int64_t j = begin - kMtN + t;
        const uint32_t v = init[t];
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

__global__ __launch_bounds__(256) void k_mt_words(uint32_t *R, int64_t begin, int64_t end) {
    mt_words_body(R, begin, end, R + begin - kMtN);
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
// The draw's results, also into the host's copy (mapped, coherent host memory)
// when given: no result copy follows the draw (a copy is a blit kernel that
// competes with the candidate pass).
__global__ __launch_bounds__(256) void k_mt_final(const uint32_t *R, int64_t pos0, int64_t b_in, int64_t P,
                                                  MtMeta *meta, MtMeta *meta_host) {
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
    if (!meta_host) return;
    __syncthreads();
    static_assert(sizeof(MtMeta) % 4 == 0, "MtMeta words");
    const uint32_t *src = reinterpret_cast<const uint32_t *>(meta);
    uint32_t *dst = reinterpret_cast<uint32_t *>(meta_host);
    for (int k = threadIdx.x; k < (int)(sizeof(MtMeta) / 4); k += 256) dst[k] = src[k];
}

__global__ __launch_bounds__(256) void k_mt_patch(double *out, const int64_t *idx, const double *val, int64_t n) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < n && idx[k] >= 0) out[idx[k]] = val[k];
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
                          MtMeta *meta_host, hipStream_t s) {
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
    hipLaunchKernelGGL(k_mt_final, dim3(1), dim3(256), 0, s, R, pos0, b_in, P, meta, meta_host);
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

// ---------------------------------------------------------------------------
// Jump-ahead: several workgroups make one draw's words.  Every bit sequence of
// the stream (bit k of x[n + 1], n >= 0) satisfies the recurrence whose
// characteristic polynomial phi (degree 19937) is that of the state transition,
// so with g = x^J mod phi, x[J + w] = XOR_{i : g_i = 1} x[i + w] for w >= 1: the
// 624 words after index J are a GF(2) combination of the first 20 561 words.
// phi is found once by Berlekamp-Massey on 2 x 19937 bits of a stream; the
// polynomials of the region starts J_k = k J are made by products mod phi.
namespace fs2 {
namespace {

constexpr int kMtDeg = 19937;
constexpr int kPW = (kMtDeg + 1 + 63) / 64;       // words of a polynomial of degree <= 19937

typedef std::vector<uint64_t> Poly;

inline int pbit(const uint64_t *p, int64_t i) { return (int)((p[i >> 6] >> (i & 63)) & 1u); }

// q ^= p << sh (q has room)
inline void xor_shifted(uint64_t *q, const uint64_t *p, int np, int64_t sh) {
    const int64_t ws = sh >> 6;
    const int bs = (int)(sh & 63);
    if (bs == 0) {
        for (int k = 0; k < np; ++k) q[k + ws] ^= p[k];
    } else {
        uint64_t carry = 0;
        for (int k = 0; k < np; ++k) {
            q[k + ws] ^= (p[k] << bs) | carry;
            carry = p[k] >> (64 - bs);
        }
        q[np + ws] ^= carry;
    }
}

// The stream's characteristic polynomial (degree 19937, bit i = coefficient of x^i).
const Poly &mt_charpoly() {
    static const Poly phi = [] {
        // a stream from an arbitrary key: MSB of x[n + 1], n = 0 .. 2 x 19937 + 63
        const int64_t nb = 2 * (int64_t)kMtDeg + 64;
        std::vector<uint32_t> x(nb + kMtN + 2);
        for (int i = 0; i < kMtN; ++i) x[i] = 0x9e3779b9u * (uint32_t)(i + 1) ^ 0x7f4a7c15u;
        for (int64_t n = kMtN; n < (int64_t)x.size(); ++n) x[n] = mt_next_word(x[n - 624], x[n - 623], x[n - 227]);
        // reversed sequence bitset: bit j = s[nb - 1 - j]
        const int nw = (int)((nb + 63) / 64) + 2;
        std::vector<uint64_t> rev(nw + kPW + 2, 0);
        for (int64_t n = 0; n < nb; ++n)
            if ((x[n + 1] >> 31) & 1u) {
                const int64_t j = nb - 1 - n;
                rev[j >> 6] |= 1ull << (j & 63);
            }
        // Berlekamp-Massey over GF(2): connection polynomial C (bit i = c_i)
        const int cw = kPW + 2;
        std::vector<uint64_t> C(cw + kPW + 4, 0), B(cw + kPW + 4, 0), T;
        C[0] = B[0] = 1;
        int64_t L = 0, m = 1;
        for (int64_t n = 0; n < nb; ++n) {
            // d = parity(C & (rev >> t)), t = nb - 1 - n: s[n] + sum c_i s[n - i]
            const int64_t t = nb - 1 - n, tw = t >> 6;
            const int tb = (int)(t & 63);
            const int lw = (int)(L >> 6) + 1;
            uint64_t acc = 0;
            for (int k = 0; k < lw; ++k) {
                const uint64_t lo = rev[tw + k], hi = rev[tw + k + 1];
                const uint64_t wv = tb ? ((lo >> tb) | (hi << (64 - tb))) : lo;
                acc ^= C[k] & wv;
            }
            if (!__builtin_parityll(acc)) {
                ++m;
            } else if (2 * L <= n) {
                T = C;
                xor_shifted(C.data(), B.data(), cw, m);
                L = n + 1 - L;
                B = T;
                m = 1;
            } else {
                xor_shifted(C.data(), B.data(), cw, m);
                ++m;
            }
        }
        // phi(x) = x^L C(1/x)
        Poly p(kPW, 0);
        for (int64_t i = 0; i <= L; ++i)
            if (pbit(C.data(), i)) {
                const int64_t j = L - i;
                p[j >> 6] |= 1ull << (j & 63);
            }
        if (L != kMtDeg) p.clear();            // (checked by the caller)
        return p;
    }();
    return phi;
}

// r (2 kPW words, degree < 2 x 19937) mod phi -> kPW words
void reduce_mod(std::vector<uint64_t> &r, const Poly &phi) {
    for (int64_t d = 2 * (int64_t)kMtDeg; d >= kMtDeg; --d)
        if (pbit(r.data(), d)) xor_shifted(r.data(), phi.data(), kPW, d - kMtDeg);
    r.resize(kPW);
}

Poly mulmod(const Poly &a, const Poly &b, const Poly &phi) {
    std::vector<uint64_t> r(2 * kPW + 2, 0);
    for (int64_t i = 0; i < kMtDeg; ++i)
        if (pbit(a.data(), i)) xor_shifted(r.data(), b.data(), kPW, i);
    reduce_mod(r, phi);
    return r;
}

Poly xpow_mod(uint64_t J, const Poly &phi) {
    Poly r(kPW, 0);
    r[0] = 1;
    int top = 63;
    while (top > 0 && !((J >> top) & 1u)) --top;
    for (int bt = top; bt >= 0; --bt) {
        // square: spread the bits
        std::vector<uint64_t> s(2 * kPW + 2, 0);
        for (int64_t i = 0; i < kMtDeg; ++i)
            if (pbit(r.data(), i)) s[(2 * i) >> 6] |= 1ull << ((2 * i) & 63);
        reduce_mod(s, phi);
        r = s;
        if ((J >> bt) & 1u) {
            std::vector<uint64_t> t(2 * kPW + 2, 0);
            xor_shifted(t.data(), r.data(), kPW, 1);
            reduce_mod(t, phi);
            r = t;
        }
    }
    return r;
}

}  // namespace

// the jump polynomials of J, 2J, ..., (G-1)J: [G-1][kPW] words into out (false: no phi)
bool mt_jump_polys(uint64_t J, int G, std::vector<uint64_t> &out) {
    const Poly &phi = mt_charpoly();
    if (phi.empty()) return false;
    out.assign((size_t)(G - 1) * kPW, 0);
    Poly g1 = xpow_mod(J, phi), gk = g1;
    for (int k = 1; k < G; ++k) {
        if (k > 1) gk = mulmod(gk, g1, phi);
        std::copy(gk.begin(), gk.end(), out.begin() + (size_t)(k - 1) * kPW);
    }
    return true;
}
int mt_poly_words() { return kPW; }

// host: x[J + 1 .. J + 624] from the key x[0 .. 624) (the device kernels' arithmetic)
bool mt_jump_host(const uint32_t key[624], uint64_t J, uint32_t out[624]) {
    std::vector<uint64_t> g;
    if (!mt_jump_polys(J, 2, g)) return false;
    std::vector<uint32_t> x(kMtDeg + kMtN + 1);
    for (int i = 0; i < kMtN; ++i) x[i] = key[i];
    for (size_t n = kMtN; n < x.size(); ++n) x[n] = mt_next_word(x[n - 624], x[n - 623], x[n - 227]);
    for (int w = 1; w <= kMtN; ++w) {
        uint32_t acc = 0;
        for (int i = 0; i < kMtDeg; ++i)
            if (pbit(g.data(), i)) acc ^= x[i + w];
        out[w - 1] = acc;
    }
    return true;
}

// ---- device side ----
constexpr int kMtJumpChunk = 1024;
constexpr int kMtBaseWords = kMtDeg + kMtN + 1;    // x[0 .. 20561): the jump's operands

// windows[k - 1][w - 1] ^= XOR over the chunk's i with g_k bit i of x[i + w]
// (grid: chunks x (G - 1); windows zeroed first)
__global__ __launch_bounds__(640) void k_mt_jump(const uint32_t *R, const uint64_t *g, int pw, uint32_t *win) {
    __shared__ uint32_t xs[kMtJumpChunk + kMtN + 1];
    __shared__ uint64_t gs[kMtJumpChunk / 64];
    const int k = blockIdx.y;
    const int i0 = blockIdx.x * kMtJumpChunk;
    for (int t = threadIdx.x; t < kMtJumpChunk + kMtN + 1; t += blockDim.x) {
        const int i = i0 + t;
        xs[t] = i < kMtBaseWords ? R[i] : 0u;
    }
    if (threadIdx.x < kMtJumpChunk / 64) {
        const int wi = (i0 >> 6) + threadIdx.x;
        gs[threadIdx.x] = wi < pw ? g[(int64_t)k * pw + wi] : 0ull;
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t >= kMtN) return;
    const int w = t + 1;
    const int n = min(kMtJumpChunk, kMtDeg - i0);
    uint32_t acc = 0;
    for (int i = 0; i < n; ++i) {
        const uint32_t m = 0u - (uint32_t)((gs[i >> 6] >> (i & 63)) & 1ull);
        acc ^= xs[i + w] & m;
    }
    atomicXor(win + (int64_t)k * kMtN + t, acc);
}

struct MtRegions {
    int64_t begin[kMtMaxGen], end[kMtMaxGen];
    int32_t from_win[kMtMaxGen];     // block k > 0: its first 624 words are window k - 1
};

// block b makes R[begin[b], end[b]) from the 624 words before begin[b] (window
// b - 1 when from_win, stored into R as well)
__global__ __launch_bounds__(256) void k_mt_words_multi(uint32_t *R, const uint32_t *win, const MtRegions rg) {
    const int b = blockIdx.x;
    const int64_t begin = rg.begin[b], end = rg.end[b];
    const uint32_t *init = R + begin - kMtN;
    if (rg.from_win[b]) {
        init = win + (int64_t)(b - 1) * kMtN;
        for (int t = threadIdx.x; t < kMtN; t += 256) R[begin - kMtN + t] = init[t];
    }
    mt_words_body(R, begin, end, init);
}

hipError_t launch_mt_words_parallel(uint32_t *R, int64_t total, const uint64_t *g, int pw, int G, int64_t J,
                                    uint32_t *win, hipStream_t s) {
    // base words for the jumps, then the G - 1 windows, then the regions
    hipError_t e = launch_mt_words(R, kMtN, kMtBaseWords, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(win, 0, sizeof(uint32_t) * kMtN * (G - 1), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mt_jump, dim3((kMtDeg + kMtJumpChunk - 1) / kMtJumpChunk, G - 1), dim3(640), 0, s, R, g,
                       pw, win);
    MtRegions rg{};
    for (int b = 0; b < G; ++b) {
        const int64_t st = b == 0 ? kMtBaseWords : (int64_t)b * (int64_t)J + 1 + kMtN;   // after window b - 1
        rg.begin[b] = st;
        rg.end[b] = b + 1 < G ? (int64_t)(b + 1) * (int64_t)J + 1 : total;
        rg.from_win[b] = b > 0;
    }
    hipLaunchKernelGGL(k_mt_words_multi, dim3(G), dim3(256), 0, s, R, win, rg);
    return hipGetLastError();
}

}  // namespace fs2
