// fs2_resample.hip -- N_eff / estimate / low-variance resampling on gfx950
// (reference fast_slam_2/algorithms/fast_slam_2.py:57-67, 177-223), for one
// GPU or for particles sharded over G ranks.
//
// Resample plan.  With the global inclusive prefix c of the normalised weights
// and u_m = u0 + m * (1/N) (evaluated exactly as the reference writes it),
// output m is a copy of the smallest particle i with c_i >= u_m (N-1 when u_m
// exceeds every prefix: the reference would loop forever there).
// Equivalently particle i fills the contiguous output range
//     { m : c_{i-1} < u_m <= c_i }   (particle N-1 also every m with u_m > c_{N-2}),
// which each rank computes for its own particles from its local prefix and the
// offset O_r = sum of the normalised totals of the ranks before it.  Outputs
// are owned by the rank holding the same global index, so a particle moves
// between ranks only when its range crosses a shard boundary.
//
// Maps move only where they must: the first local output of a local source
// keeps the source's map; every other output (extra copies, particles received
// from another rank) takes over the map of a local particle that feeds no
// local output, whose landmarks were already packed if another rank needs them.
#include "fs2_chain.hpp"
#include "fs2_plan.hpp"

namespace fs2 {

constexpr int kScanPer = 4;                       // elements per thread
constexpr int kScanBlock = kBlock * kScanPer;     // 1024 elements per block

// ------------------------------------------------------- global reductions --

// Weight total over ranks, in shard order (world > 1; totals are gathered by rank).
__global__ void k_global_total(const ReduceParams P) {
    double t = 0.0;
    for (int q = 0; q < P.world; ++q) {
        if (q == P.shard && P.est_base) *P.est_base = t;     // sharded exact: the chain's estimate base
        t = (q == 0) ? P.totals[P.rank_of[0]] : t + P.totals[P.rank_of[q]];
    }
    P.stats->total = t;
}

hipError_t launch_global_total(const ReduceParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_global_total, dim3(1), dim3(1), 0, s, p);
    return hipGetLastError();
}

// numpy pairwise summation of w[i]^2 (loops_utils.h.src) for the sequential mode.
__device__ double pairwise_sq(const double *a, int64_t n) {
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
    return pairwise_sq(a, n2) + pairwise_sq(a + n2, n - n2);
}

template <typename RecOf>
__device__ void global_finalize_impl(const ReduceParams &P, RecOf rec, const double *sq_exact = nullptr);

// This rank's record: sum w'^2, first maximum, its pose, normalised total (on
// one GPU also the global decision, k_global_finalize's work).
constexpr int kNpStage = 1024;

// Optional phase stamps of k_finalize (build with -DFS2_PHASE_TIMING; read back
// with fs2_debug_finalize_times): thread 0's s_memtime deltas, summed.
#ifdef FS2_PHASE_TIMING
__device__ unsigned long long g_fin[8];
#define FS2_FIN(k)                                                                   \
    do {                                                                             \
        if (threadIdx.x == 0) {                                                      \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();               \
            if ((k) > 0) atomicAdd(&g_fin[(k) - 1], t_ - fin_last);                 \
            fin_last = t_;                                                           \
        }                                                                            \
    } while (0)
#else
#define FS2_FIN(k) do { } while (0)
#endif

__device__ void publish_body(DevStats *stats, DevStats *host_stats, unsigned long long *host_flag,
                             unsigned long long seq);

__global__ __launch_bounds__(1024) void k_finalize(const ReduceParams P) {
    __shared__ int s_kept;
    __shared__ double lds_d[16];
    __shared__ int64_t lds_l[16];
    __shared__ int lds_i[16];
    __shared__ double s_np[kNpStage];
    __shared__ double s_bv[16];
#ifdef FS2_PHASE_TIMING
    unsigned long long fin_last = 0;
#endif
    FS2_FIN(0);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the normalise partials: every thread's loads issued first, so that their
    // latency overlaps the numpy trees below
    constexpr int PL = 4;
    double s4[PL], w4[PL], t4[PL];
    int64_t i4[PL];
    int m4[PL];
    double sq = 0.0, tw = 0.0;
    __shared__ double s_tw, lds_t[16];
    double bv = -INFINITY;
    int64_t bi = INT64_MAX;
    int mc = 0;
    auto load_parts = [&](int k0) {
#pragma unroll
        for (int u = 0; u < PL; ++u) {
            const int k = k0 + 1024 * u;
            const bool in = k < P.nparts;
            s4[u] = in ? P.part_sq[k] : 0.0;
            t4[u] = (in && P.t_from_parts) ? P.part_w[k] : 0.0;
            w4[u] = in ? P.part_best_w[k] : -INFINITY;
            i4[u] = in ? P.part_best_i[k] : INT64_MAX;
            m4[u] = in ? P.part_maxcnt[k] : 0;
        }
    };
    auto fold_parts = [&] {
#pragma unroll
        for (int u = 0; u < PL; ++u) {
            sq += s4[u];
            tw += t4[u];
            argmax_combine(bv, bi, w4[u], i4[u]);
            mc = max(mc, m4[u]);
        }
    };
    load_parts(threadIdx.x);
    if (P.exact) {
        // numpy's chunk sums: each full chunk's 64 leaves (k_normalize) as a balanced
        // tree in order (a wave per chunk, xor butterflies; 16 chunks' loads in
        // flight) on waves 0..14, the partial last chunk by numpy's recursion on
        // wave 15 meanwhile; added in order by thread 0 below
        const int64_t nfull = P.n / kNpChunk;
        if (wid < 15) {
            for (int64_t c0 = wid; c0 < nfull; c0 += 15 * 16) {
                double v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int64_t c = c0 + 15 * u;
                    v[u] = (c < nfull) ? P.np_leaf[c * 64 + lane] : 0.0;
                }
                // the DPP reduction's tree is numpy's: row_shr 1/2/4/8 pair the
                // leaves of each 16-lane row as a balanced tree in order (the adds
                // commute), the row broadcasts then pair rows 0+1, 2+3 and the halves
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    v[u] = lane63(dpp_scan(v[u], 0.0, [](double a, double b) { return a + b; }));
                    const int64_t c = c0 + 15 * u;
                    if (lane == 0 && c < nfull) {
                        if (c < kNpStage) s_np[c] = v[u];
                        else P.np_part[c] = v[u];
                    }
                }
            }
        } else if (P.np_tail) {
            const double t = np_pairwise_wave(P.w + nfull * kNpChunk, P.np_tail);
            if (lane == 0) {
                if (nfull < kNpStage) s_np[nfull] = t;
                else P.np_part[nfull] = t;
            }
        }
    }
    FS2_FIN(1);
    fold_parts();
    for (int k0 = threadIdx.x + PL * 1024; k0 < P.nparts; k0 += PL * 1024) {
        load_parts(k0);
        fold_parts();
    }
    FS2_FIN(2);
    // the three block reductions behind one barrier (wave trees on DPP)
    sq = wave_sum(sq);
    tw = wave_sum(tw);
    wave_argmax(bv, bi);
    mc = wave_max_i(mc);
    if (lane == 0) {
        lds_t[wid] = tw;
        lds_d[wid] = sq;
        s_bv[wid] = bv;
        lds_l[wid] = bi;
        lds_i[wid] = mc;
    }
    __syncthreads();
    FS2_FIN(3);
    if (threadIdx.x == 0) {
        sq = lds_d[0];
        bv = s_bv[0];
        bi = lds_l[0];
        mc = lds_i[0];
        tw = lds_t[0];
#pragma unroll
        for (int k = 1; k < 16; ++k) {
            sq += lds_d[k];
            tw += lds_t[k];
            argmax_combine(bv, bi, s_bv[k], lds_l[k]);
            mc = max(mc, lds_i[k]);
        }
        s_tw = tw;
    }
    FS2_FIN(4);
    if (threadIdx.x == 0) {
        if (P.sequential) {
            // np.sum(weights ** 2): pairwise inside 8192-element chunks
            double s = 0.0;
            for (int64_t k = 0; k < P.n; k += 8192) {
                const int64_t m = (P.n - k < 8192) ? P.n - k : 8192;
                const double p = pairwise_sq(P.w + k, m);
                s = (k == 0) ? p : s + p;
            }
            sq = s;
        } else if (P.exact) {
            // the same sums: each chunk's tree (above), added in order
            // (the LDS-staged ones first: one address space per loop, so the loads
            // stay ds_read instead of flat)
            const int nl = min(P.n_np, kNpStage);
            double s = (nl > 0) ? s_np[0] : 0.0;
            for (int k = 1; k < nl; ++k) s = s + s_np[k];
            for (int k = nl; k < P.n_np; ++k) s = s + P.np_part[k];
            sq = s;
        }
        FS2_FIN(5);
        RankRecord r{};
        r.sumsq = sq;
        r.best_w = bv;
        r.best_gidx = (bi == INT64_MAX) ? INT64_MAX : P.gidx0 + bi;
        if (bi != INT64_MAX) {
            r.pose[0] = P.x[bi];
            r.pose[1] = P.y[bi];
            r.pose[2] = P.yaw[bi];
        }
        r.t_local = P.stats->t_local;
        // sharded exact mode: a tree estimate of this shard's normalised total (the
        // resample chain's estimate base; no local prefix is formed)
        if (P.t_from_parts) r.t_local = s_tw;
        r.max_count = mc;
        r.want_collect = P.want_collect;
        *P.rec = r;
        FS2_FIN(6);
        // one GPU: no record exchange (the record from registers)
        if (P.world == 1 && P.recs == P.rec) global_finalize_impl(P, [&](int) -> const RankRecord & { return r; });
        FS2_FIN(7);
        if (threadIdx.x == 0) {
#ifdef FS2_PHASE_TIMING
            atomicAdd(&g_fin[7], 1ull);
#endif
        }
        s_kept = (P.pub_flag != nullptr && !P.stats->resampled) ? 1 : 0;
    }
    // one GPU, rule not fired: the scan is complete, publish it now (the lazy
    // resample kernels then run while the host returns and enqueues the next scan)
    __syncthreads();
    if (s_kept) publish_body(P.stats, P.pub_host, P.pub_flag, P.pub_seq);
}

#ifdef FS2_PHASE_TIMING
FS2_TAIL_READER(debug_tail_times_resample)
hipError_t debug_fin_times(unsigned long long out[8], int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fin), sizeof(unsigned long long) * 8);
    if (e == hipSuccess && reset) {
        unsigned long long z[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_fin), z, sizeof z);
    }
    return e;
}
#endif

// One GPU, exact mode, after k_normalize_chunks: its partials (half-chunk sums
// of numpy's Sigma w'^2, first maxima with their poses, largest maps) folded by
// one wave -- no workgroup barrier, no dependent load -- then the same record,
// decision, estimate and u0 as k_finalize (fast_slam_2.py:60-67, 201-223), and the
// publication when the rule did not fire.
__global__ __launch_bounds__(64) void k_finalize_chunked(const ReduceParams P) {
    __shared__ double s_np[kNpStage];
    FS2_TS_DECL;
    FS2_TS(24, 0);
    const int lane = threadIdx.x;
    double bv = -INFINITY, px = 0.0, py = 0.0, pyaw = 0.0;
    int64_t bi = INT64_MAX;
    int mc = 0;
    // np.sum's full chunks (numpy's top node: half 2c + half 2c + 1), one per lane and
    // register, loaded with the partials below and added in order from registers
    // (readlane) by the whole wave: no LDS round trip per step of the serial sum
    const int64_t nfull = P.n / kNpChunk;
    const bool creg = nfull <= 128;
    double cv[2] = {0.0, 0.0};
    if (creg) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int64_t c = lane + 64 * j;
            if (c < nfull) cv[j] = P.np_part[2 * c] + P.np_part[2 * c + 1];
        }
    }
    for (int k0 = 0; k0 < P.nparts; k0 += 256) {
        double w4[4], x4[4], y4[4], a4[4], s4[4];
        int64_t i4[4];
        int m4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + 64 * u + lane;
            const bool in = k < P.nparts;
            w4[u] = in ? P.part_best_w[k] : -INFINITY;
            i4[u] = in ? P.part_best_i[k] : INT64_MAX;
            m4[u] = in ? P.part_maxcnt[k] : 0;
            s4[u] = in ? P.np_part[k] : 0.0;
            x4[u] = in ? P.part_pose[3 * (int64_t)k] : 0.0;
            y4[u] = in ? P.part_pose[3 * (int64_t)k + 1] : 0.0;
            a4[u] = in ? P.part_pose[3 * (int64_t)k + 2] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + 64 * u + lane;
            if (w4[u] > bv || (w4[u] == bv && i4[u] < bi)) {
                bv = w4[u];
                bi = i4[u];
                px = x4[u];
                py = y4[u];
                pyaw = a4[u];
            }
            mc = max(mc, m4[u]);
            if (k < P.nparts && k < kNpStage) s_np[k] = s4[u];
        }
    }
    FS2_TS(24, 1);
    // first maximum over the wave, its pose carried along (lowest index on ties)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double v2 = __shfl_xor(bv, o, 64), x2 = __shfl_xor(px, o, 64), y2 = __shfl_xor(py, o, 64),
                     a2 = __shfl_xor(pyaw, o, 64);
        const int64_t i2 = __shfl_xor(bi, o, 64);
        if (v2 > bv || (v2 == bv && i2 < bi)) {
            bv = v2;
            bi = i2;
            px = x2;
            py = y2;
            pyaw = a2;
        }
    }
    mc = wave_max_i(mc);
    // the full chunks' sums in order (wave-uniform: every lane adds the same values)
    double sqr = 0.0;
    if (creg) {
        const int n0 = (int)min<int64_t>(nfull, 64);
        for (int c = 0; c < n0; ++c) {
            const double v = bcast(cv[0], c);
            sqr = (c == 0) ? v : sqr + v;
        }
        for (int c = 64; c < (int)nfull; ++c) sqr = sqr + bcast(cv[1], c - 64);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    __shared__ int s_kept;
    if (lane == 0) {
        // np.sum(weights ** 2): chunk c = half 2c + half 2c + 1 (numpy's top node),
        // a partial last chunk whole; the chunk sums in order
        auto part = [&](int64_t k) -> double { return k < kNpStage ? s_np[k] : P.np_part[k]; };
        double sq = sqr;
        if (!creg) {
            for (int64_t c = 0; c < nfull; ++c) {
                const double v = part(2 * c) + part(2 * c + 1);
                sq = (c == 0) ? v : sq + v;
            }
        }
        if (P.n % kNpChunk) sq = (nfull == 0) ? part(2 * nfull) : sq + part(2 * nfull);
        RankRecord r{};
        r.sumsq = sq;
        r.best_w = bv;
        r.best_gidx = (bi == INT64_MAX) ? INT64_MAX : P.gidx0 + bi;
        r.pose[0] = px;
        r.pose[1] = py;
        r.pose[2] = pyaw;
        r.t_local = P.stats->t_local;
        r.max_count = mc;
        *P.rec = r;
        global_finalize_impl(P, [&](int) -> const RankRecord & { return r; });
        s_kept = (P.pub_flag != nullptr && !P.stats->resampled) ? 1 : 0;
    }
    FS2_TS(24, 2);
    __syncthreads();
    if (s_kept) publish_body(P.stats, P.pub_host, P.pub_flag, P.pub_seq);
    FS2_TS(24, 3);
}

hipError_t launch_finalize_chunked(const ReduceParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize_chunked, dim3(1), dim3(64), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_finalize(const ReduceParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

// N_eff (fast_slam_2.py:212-223), the N_eff < N/2 rule (:62), the estimate
// (:201-210), u0 (:183) and this rank's prefix offset, from all records (held
// by rank; the sums run in shard order, the first maximum is order-free).
template <typename RecOf>
__device__ void global_finalize_impl(const ReduceParams &P, RecOf rec, const double *sq_exact) {
    DevStats *st = P.stats;
    const int g0 = P.rank_of[0];
    double sq = rec(g0).sumsq;
    double bv = rec(g0).best_w;
    int64_t bi = rec(g0).best_gidx;
    int gb = g0;
    double off = 0.0;
    for (int q = 1; q < P.world; ++q) {
        const int g = P.rank_of[q];
        sq = sq + rec(g).sumsq;
        const double v = rec(g).best_w;
        const int64_t i = rec(g).best_gidx;
        if (v > bv || (v == bv && i < bi)) {
            bv = v;
            bi = i;
            gb = g;
        }
    }
    for (int q = 0; q < P.shard; ++q) off = (q == 0) ? rec(g0).t_local : off + rec(P.rank_of[q]).t_local;
    if (sq_exact) sq = *sq_exact;
    const double ng = (double)P.n_global;
    const double ne = (sq < 1.0 / ng) ? ng : 1.0 / sq;
    st->sumsq = sq;
    st->n_eff = ne;
    // fs2.h error_flags bit 1: a weight (hence the total) is not finite; the
    // rule then never fires (NaN < N/2 is false), as in the reference
    if (!isfinite(st->total) || !isfinite(sq)) st->error_flags |= 2;
    st->resampled = ne < ng / 2.0 ? 1 : 0;
    // tree sums: a decision this close to the threshold may differ from the
    // reference's summation order
    if (P.flip_margin > 0.0 && fabs(ne - ng / 2.0) <= P.flip_margin * ng) st->reduce_amb += 1;
    // the largest map on any rank: a resample may bring it here (the receiver
    // sizes its page-table rows for it before unpacking)
    int mc = rec(0).max_count, wc = rec(0).want_collect;
    for (int g = 1; g < P.world; ++g) {
        mc = max(mc, rec(g).max_count);
        wc |= rec(g).want_collect;
    }
    st->collect_next = wc;
    st->max_count = max(st->max_count, mc);
    st->best_index = bi;
    st->best_w = bv;
    st->pose[0] = rec(gb).pose[0];
    st->pose[1] = rec(gb).pose[1];
    st->pose[2] = rec(gb).pose[2];
    st->offset = off;
    st->out_min = INT32_MAX;
    st->out_max = -1;
    st->u0 = P.u0_host ? *P.u0_host
                       : (1.0 / ng) * philox_uniform01(P.seed, P.scan | (1ull << 63), 0);
}

__global__ void k_global_finalize(const ReduceParams P) {
    global_finalize_impl(P, [&](int g) -> const RankRecord & { return P.recs[g]; });
}

// Sharded exact mode: np.sum(w'^2) over the global order (fast_slam_2.py:219) from
// every shard's chunk sums, the chunks cut by shard boundaries completed from both
// neighbours' edges (the cut leaf from their raw weights), added in order; then
// the rest of k_global_finalize.  One thread.
__global__ void k_global_finalize_x(const ReduceParams P, const RankRecordX *all, const NpTailPlan *gtail) {
    double node[2 * kNpMaxLeaves];
    double sq = 0.0;
    bool any = false;
    auto add = [&](double v) {
        sq = any ? sq + v : v;
        any = true;
    };
    for (int q = 0; q < P.world; ++q) {
        const RankRecordX &X = all[P.rank_of[q]];
        if (q > 0 && X.head.chunk >= 0) {
            const NpEdge &T = all[P.rank_of[q - 1]].tail, &H = X.head;
            const int64_t cs = (int64_t)H.chunk * kNpChunk;
            const int m = (int)min<int64_t>(kNpChunk, P.n_global - cs);
            const int nl = np_chunk_leaves(m, gtail);
            bool ok = T.chunk == H.chunk;
            for (int k = 0; k < nl; ++k) {
                if (k >= T.leaf0 && k < T.leaf0 + T.nleaf) node[k] = T.leaf[k - T.leaf0];
                else if (k >= H.leaf0 && k < H.leaf0 + H.nleaf) node[k] = H.leaf[k - H.leaf0];
                else if (k == H.cut && k == T.cut && T.nraw + H.nraw == np_leaf_len(m, gtail, k))
                    node[k] = np_leaf_seq([&](int i) { return i < T.nraw ? T.raw[i] : H.raw[i - T.nraw]; },
                                          T.nraw + H.nraw);
                else ok = false;
            }
            if (!ok) {                   // edges that do not fit together: counted, never hidden
                P.stats->reduce_amb += 1;
                P.stats->error_flags |= 4;
                node[0] = 0.0;
                for (int k = 1; k < nl; ++k) node[k] = 0.0;
            }
            add(np_chunk_combine(node, m, gtail));
        }
        for (int j = 0; j < X.nsums; ++j) add(X.sums[j]);
    }
    global_finalize_impl(P, [&](int g) -> const RankRecord & { return all[g].base; }, &sq);
}

hipError_t launch_global_finalize_x(const ReduceParams &p, const RankRecordX *all, const NpTailPlan *gtail,
                                    hipStream_t s) {
    hipLaunchKernelGGL(k_global_finalize_x, dim3(1), dim3(1), 0, s, p, all, gtail);
    return hipGetLastError();
}

hipError_t launch_global_finalize(const ReduceParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_global_finalize, dim3(1), dim3(1), 0, s, p);
    return hipGetLastError();
}

// Estimate after a resample: first maximum over all ranks' outputs.
__device__ void global_best_body(const ReduceParams &P) {
    DevStats *st = P.stats;
    double bv = P.recs[0].best_w;
    int64_t bi = P.recs[0].best_gidx;
    int gb = 0;
    for (int g = 1; g < P.world; ++g) {
        const double v = P.recs[g].best_w;
        const int64_t i = P.recs[g].best_gidx;
        if (v > bv || (v == bv && i < bi)) {
            bv = v;
            bi = i;
            gb = g;
        }
    }
    st->best_index = bi;
    st->best_w = bv;
    st->pose[0] = P.recs[gb].pose[0];
    st->pose[1] = P.recs[gb].pose[1];
    st->pose[2] = P.recs[gb].pose[2];
}

__global__ void k_global_best(const ReduceParams P) {
    if (P.stats->resampled) global_best_body(P);
}

hipError_t launch_global_best(const ReduceParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_global_best, dim3(1), dim3(1), 0, s, p);
    return hipGetLastError();
}

__device__ void publish_body(DevStats *stats, DevStats *host_stats, unsigned long long *host_flag,
                             unsigned long long seq) {
    static_assert(sizeof(DevStats) % 8 == 0 && sizeof(DevStats) / 8 <= 64, "one word per lane");
    constexpr int W = sizeof(DevStats) / 8;
    const int t = threadIdx.x;
    if (t < W) {
        uint64_t *s = reinterpret_cast<uint64_t *>(stats);
        const uint64_t v = s[t];
        reinterpret_cast<uint64_t *>(host_stats)[t] = v;
        s[t] = 0;                    // the next scan's counters start from zero
    }
    // the barrier completes every thread's stores; thread 0's system-scope release
    // (cumulative) then orders all of them before the flag -- one cache write-back,
    // not one per thread
    __syncthreads();
    if (t == 0) __hip_atomic_store(host_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void k_publish(DevStats *stats, DevStats *host_stats, unsigned long long *host_flag,
                                                unsigned long long seq) {
    publish_body(stats, host_stats, host_flag, seq);
}

// Mid-scan post (sharded ranks): the scan's statistics so far and the
// all-gathered transfer sizes into coherent host memory, then the flag; the host
// spins on it instead of a copy and a stream sync.
__global__ __launch_bounds__(256) void k_post(const DevStats *stats, const int64_t *xmat, int32_t nx, char *host,
                                              unsigned long long *host_flag, unsigned long long seq) {
    constexpr int W = sizeof(DevStats) / 8;
    const int t = threadIdx.x;
    if (t < W) reinterpret_cast<uint64_t *>(host)[t] = reinterpret_cast<const uint64_t *>(stats)[t];
    for (int k = t; k < nx; k += blockDim.x) reinterpret_cast<int64_t *>(host + sizeof(DevStats))[k] = xmat[k];
    __syncthreads();                 // then thread 0's system-scope release orders them all
    if (t == 0) __hip_atomic_store(host_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_post(const DevStats *stats, const int64_t *xmat, int32_t nx, char *host,
                       unsigned long long *host_flag, unsigned long long seq, hipStream_t s) {
    hipLaunchKernelGGL(k_post, dim3(1), dim3(256), 0, s, stats, xmat, nx, host, host_flag, seq);
    return hipGetLastError();
}

hipError_t launch_publish(DevStats *stats, DevStats *host_stats, unsigned long long *host_flag,
                          unsigned long long seq, hipStream_t s, hipEvent_t e1) {
    FS2_LAUNCH_EV(k_publish, dim3(1), dim3(64), s, nullptr, e1, stats, host_stats, host_flag, seq);
    return hipGetLastError();
}

// ------------------------------------------------------------ local prefix --

__device__ __forceinline__ double wave_incl_scan(double v) {
    return dpp_scan(v, 0.0, [](double a, double b) { return a + b; });
}

__device__ __forceinline__ int wave_incl_scan_i(int v) {
    return dpp_scan(v, 0, [](int a, int b) { return a + b; });
}

// Sequential running sum, the reference's order (fast_slam_2.py:184-193).
__global__ __launch_bounds__(1) void k_scan_seq(const ResampleParams P) {
    if (P.lazy && !P.stats->resampled) return;
    double c = 0.0;
    for (int64_t i = 0; i < P.n; ++i) {
        c = (i == 0) ? P.w[0] : c + P.w[i];
        P.c[i] = c;
    }
    P.stats->t_local = (P.n > 0) ? c : 0.0;
}

__global__ __launch_bounds__(kBlock) void k_scan_local(const ResampleParams P) {
    __shared__ double lds[kBlock / 64];
    if (P.lazy && !P.stats->resampled) return;
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanPer;
    double v[kScanPer];
    double run = 0.0;
#pragma unroll
    for (int e = 0; e < kScanPer; ++e) {
        const int64_t i = base + e;
        run += (i < P.n) ? P.w[i] : 0.0;
        v[e] = run;
    }
    const double incl = wave_incl_scan(run);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) lds[wid] = incl;
    __syncthreads();
    double woff = 0.0;
    for (int k = 0; k < wid; ++k) woff += lds[k];
    const double off = woff + incl - run;
#pragma unroll
    for (int e = 0; e < kScanPer; ++e) {
        const int64_t i = base + e;
        if (i < P.n) P.c[i] = off + v[e];
    }
    if (threadIdx.x == kBlock - 1) P.bsum[blockIdx.x] = off + v[kScanPer - 1];
}

// exclusive scan of the block sums: 1024 threads, each a contiguous run of blocks
__global__ __launch_bounds__(1024) void k_scan_blocks(const ResampleParams P) {
    __shared__ double lds[1024 / 64];
    if (P.lazy && !P.stats->resampled) return;
    const int per = (P.nblk + 1023) / 1024;
    const int b0 = threadIdx.x * per, b1 = min(P.nblk, b0 + per);
    double run = 0.0;
    for (int b = b0; b < b1; ++b) run += P.bsum[b];
    const double incl = wave_incl_scan(run);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) lds[wid] = incl;
    __syncthreads();
    double off = incl - run;
    for (int k = 0; k < wid; ++k) off += lds[k];
    for (int b = b0; b < b1; ++b) {
        const double t = P.bsum[b];
        P.bsum[b] = off;
        off += t;
    }
}

__global__ __launch_bounds__(kBlock) void k_scan_add(const ResampleParams P) {
    if (P.lazy && !P.stats->resampled) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < P.n) {
        const double v = P.c[i] + P.bsum[i / kScanBlock];
        P.c[i] = v;
        if (i == P.n - 1) P.stats->t_local = v;
    }
}

hipError_t launch_prefix(const ResampleParams &p, int sequential, hipStream_t s) {
    const unsigned g = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (g == 0) return hipSuccess;
    if (sequential) {
        hipLaunchKernelGGL(k_scan_seq, dim3(1), dim3(1), 0, s, p);
    } else {
        hipLaunchKernelGGL(k_scan_local, dim3(p.nblk), dim3(kBlock), 0, s, p);
        hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, p);
        hipLaunchKernelGGL(k_scan_add, dim3(g), dim3(kBlock), 0, s, p);
    }
    return hipGetLastError();
}

// ----------------------------------------------------------------- ranges --
// (plan arithmetic: fs2_plan.hpp, shared with the host entry points fs2_plan_*)

__global__ __launch_bounds__(kBlock) void k_ranges(const ResampleParams P) {
    if (!P.stats->resampled) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    __shared__ unsigned long long lds_u[kBlock / 64];
    __shared__ int64_t s_key[kBlock];
    int64_t llo = INT64_MAX, lhi = -1;       // this particle's local outputs
    unsigned amb = 0;
    // exact chain (one GPU): the running sum of this wave's unit from the unit
    // table -- a translation unit's values are s_in + (prefix of rint(w / u)) u,
    // a serial unit's were written by k_chain_walk (with the value before it)
    double cv = 0.0, cprev = 0.0;
    if (P.use_chain) {
        const int64_t k = i / kUnit;
        const int32_t info = (k * kUnit < P.n) ? P.chain.uinfo[k] : 1;
        if (info & 1) {
            cv = (i < P.n) ? P.c[i] : 0.0;
            // (a sharded rank's first element: the chain value before it, k_chain_fold)
            cprev = (i > 0 && i - 1 < P.n) ? P.c[i - 1] : (i == 0 && P.a > 0 ? P.stats->offset : 0.0);
        } else {
            // (an identity unit adds 0 and inherits the run's binade)
            const bool idu = (info & 2) != 0;
            const int E = unit_binade(info);
            const double u = unit_ulp(E);
            const double s_in = chain_unit_entry(P.chain, k, (idu && k > 0) ? chain_elast(P.chain.uel, P.chain.bpe, k - 1) : E);
            const long long r = (i < P.n && !idu) ? (long long)rint(scaled(P.w[i], E)) : 0;
            const long long pre = wave_incl_scan_i64(r);
            cv = s_in + (double)pre * u;
            cprev = s_in + (double)(pre - r) * u;
        }
    }
    if (i < P.n) {
        const double u0 = P.stats->u0, off = P.stats->offset;
        const int64_t g = P.a + i;
        const double cur = P.use_chain ? cv : ((P.a == 0) ? P.c[i] : off + P.c[i]);
        const double prev = (g == 0) ? 0.0
                                     : (P.use_chain ? cprev
                                                    : ((i == 0) ? off : ((P.a == 0) ? P.c[i - 1] : off + P.c[i - 1])));
        int64_t lo, hi;
        plan_range(g, P.N, prev, cur, u0, lo, hi);
        if (P.ranges_mode & 1) {
            P.mlo[i] = (int32_t)lo;
            P.mhi[i] = (int32_t)hi;
        }
        // tree prefix: a u_m within the rounding bound of this boundary might fall
        // on the other side of the reference's sequential value
        if ((P.ranges_mode & 1) && P.flip_margin > 0.0 && g != P.N - 1) {
            const int64_t m1 = hi + 1;                  // first output with u > cur
            const double tol = P.flip_margin * cur;
            if ((m1 < P.N && plan_u(u0, m1, P.N) - cur <= tol) || (m1 > 0 && cur - plan_u(u0, m1 - 1, P.N) <= tol))
                amb = 1;
        }
        llo = max(lo, P.ao);
        lhi = min(hi, P.ao + P.n - 1);
    }
    if (!(P.ranges_mode & 2)) llo = INT64_MAX;     // ranges only: no output filled here
    // out_src of the local outputs.  The wave's sources are consecutive and their
    // local output ranges partition one contiguous range in order, so the wave
    // fills that range together, 64 outputs per step (one lane per source would
    // store a heavy source's outputs one by one): output o comes from the last
    // lane whose key <= o, key = the first local output of the lane or, for a lane
    // with none, of the next lane that has some (a suffix minimum, non-decreasing).
    {
        const int lane = threadIdx.x & 63;
        const bool has = llo <= lhi;
        int64_t key = has ? llo : INT64_MAX;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t t = __shfl_down(key, o, 64);
            if (lane + o < 64) key = min(key, t);
        }
        s_key[threadIdx.x] = key;
        int64_t wlo = has ? llo : INT64_MAX, whi = has ? lhi : -1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            wlo = min(wlo, (int64_t)__shfl_xor(wlo, o, 64));
            whi = max(whi, (int64_t)__shfl_xor(whi, o, 64));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int64_t *wk = s_key + (threadIdx.x - lane);
        // A wave with more than kWaveFill outputs (heavy sources: the siblings of a
        // good ancestor sit side by side, so one wave can hold 64 sources of ~2000
        // outputs each -- 700 us for that wave alone in a collapsed resample) lists its
        // runs, cut into kFillChunk pieces, for k_fill_runs, where every workgroup
        // takes pieces; a full list leaves the rest of the wave's runs to the wave.
        bool listed = false;
        if (wlo <= whi && whi - wlo + 1 > kWaveFill && P.runs) {
            const bool mine = llo <= lhi;
            const int64_t pieces = mine ? (lhi - llo + kFillChunk) / kFillChunk : 0;
            const uint32_t base = pieces ? atomicAdd(P.runs_n, (uint32_t)pieces) : 0u;
            const bool fits = !mine || base + (uint64_t)pieces <= (uint64_t)kMaxLongRuns;
            // every slot below the list's end that this lane took is written (k_fill_runs
            // reads all of them), a lane that did not fit whole included
            for (int64_t q = 0; q < pieces && base + (uint64_t)q < (uint64_t)kMaxLongRuns; ++q) {
                const int64_t a = llo + q * kFillChunk, b = min(lhi, a + kFillChunk - 1);
                P.runs[base + q] = make_int4((int)(a - P.ao), (int)(b - P.ao), (int)i, 0);
            }
            listed = __ballot(!fits) == 0ull;
        }
#ifdef FS2_AB_NO_FILL
        listed = true;                // (timing probe only: out_src left unfilled)
#endif
        // otherwise the wave fills its outputs 64 per step
        // (a wave without local outputs has wlo = INT64_MAX: no step)
        for (int64_t o = (!listed && wlo <= whi) ? wlo + lane : INT64_MAX; o <= whi; o += 64) {
            int l = 0, h = 63;
            while (l < h) {
                const int mid = (l + h + 1) >> 1;
                if (wk[mid] <= o) l = mid;
                else h = mid - 1;
            }
            P.out_src[o - P.ao] = (int32_t)(i - lane + l);
        }
    }
    if (P.flip_margin > 0.0) {
        const unsigned long long ba = block_sum_u64<kBlock>(amb, lds_u);
        if (threadIdx.x == 0 && ba) atomicAdd(&P.stats->reduce_amb, ba);
        __syncthreads();             // lds_u is reused below
    }
    if (P.est_early) {
        // the outputs' first maximum (fast_slam_2.py:201-210 after :196): outputs are
        // in source order and copy their source's weight, so it is the first output
        // of the first heaviest source that has outputs; and the slots they refer to.
        // The key carries the source (output << 32 | source): its outputs may sit in
        // a listed run that k_tail_single's other workgroups fill meanwhile
        __shared__ double lds_d[kBlock / 64];
        __shared__ int64_t lds_l[kBlock / 64];
        const bool has = i < P.n && llo <= lhi;
        double bv = has ? P.w[i] : -INFINITY;
        int64_t bi = has ? ((llo - P.ao) << 32) | i : INT64_MAX;
        const unsigned long long sl = has ? (unsigned long long)(lhi - llo + 1) * (unsigned long long)P.cnt[i] : 0ull;
        const unsigned long long bs = block_sum_u64<kBlock>(sl, lds_u);
        block_argmax<kBlock>(bv, bi, lds_d, lds_l);
        if (threadIdx.x == 0) {
            P.part_best_w[blockIdx.x] = bv;
            P.part_best_i[blockIdx.x] = bi;
            P.part_slots[blockIdx.x] = bs;
        }
    }
}

// The pieces k_ranges listed (at most kFillChunk outputs each, all naming one
// source): one workgroup per piece at a time.  Lazy like k_ranges: nothing listed,
// nothing done.
__device__ __forceinline__ void fill_runs_body(const ResampleParams &P, uint32_t b, uint32_t nb) {
    const uint32_t nr = min(*P.runs_n, (uint32_t)kMaxLongRuns);
    for (uint32_t r = b; r < nr; r += nb) {
        const int4 run = P.runs[r];
        for (int64_t o = run.x + (int64_t)threadIdx.x; o <= run.y; o += blockDim.x) P.out_src[o] = run.z;
    }
}

__global__ __launch_bounds__(kBlock) void k_fill_runs(const ResampleParams P) {
    fill_runs_body(P, blockIdx.x, gridDim.x);
}

hipError_t launch_resample_ranges(const ResampleParams &p, hipStream_t s, bool fill_runs) {
    const unsigned g = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ranges, dim3(g), dim3(kBlock), 0, s, p);
    if (fill_runs && (p.ranges_mode & 2) && p.runs)
        hipLaunchKernelGGL(k_fill_runs, dim3(std::min<unsigned>(g, 256u)), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

// ------------------------------------------------- packing for other ranks --
//
// The local particles whose outputs reach rank p form one run [i0_p, i1_p) of
// the local index (fs2_plan.hpp plan_run), so one exclusive count E of the
// non-empty ranges and one of their page-table rows C serve every destination:
// the particle at i is header E[i] - E[i0_p] of rank p's transfer and its row
// entries start at C[i] - C[i0_p].  The rows name pages, sent once per
// destination however many particles name them (k_dedup_*: siblings of one
// resample share every page neither has written since).  No host round trip
// per destination: the sizes go to every rank in all-gathers of xrow.

// E, C (page-table rows) inside each 1024-particle block (rank_d, rank_e) and per-block totals
// (iblk[b], iblk[nblk + b]); lanes past n count nothing.
__global__ __launch_bounds__(kBlock) void k_pack_plan(const ResampleParams P) {
    __shared__ long long lds[2][kBlock / 64];
    if (!P.stats->resampled) return;
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanPer;
    int fa[kScanPer];
    long long fb[kScanPer];
    long long sa = 0, sb = 0;
#pragma unroll
    for (int e = 0; e < kScanPer; ++e) {
        const int64_t t = base + e;
        fa[e] = 0;
        fb[e] = 0;
        if (t < P.n && P.mlo[t] <= P.mhi[t]) {
            fa[e] = 1;
            fb[e] = (P.cnt[t] + kPageSlots - 1) / kPageSlots;
        }
        sa += fa[e];
        sb += fb[e];
    }
    const long long ia = wave_incl_scan_i64(sa), ib = wave_incl_scan_i64(sb);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) {
        lds[0][wid] = ia;
        lds[1][wid] = ib;
    }
    __syncthreads();
    long long oa = ia - sa, ob = ib - sb;
    for (int k = 0; k < wid; ++k) {
        oa += lds[0][k];
        ob += lds[1][k];
    }
#pragma unroll
    for (int e = 0; e < kScanPer; ++e) {
        const int64_t t = base + e;
        if (t < P.n) {
            P.rank_d[t] = (int32_t)oa;          // < 1024
            P.rank_e[t] = (int32_t)ob;          // < 1024 * kMaxRows
        }
        oa += fa[e];
        ob += fb[e];
    }
    if (threadIdx.x == kBlock - 1) {
        P.iblk[blockIdx.x] = oa;
        P.iblk[P.nblk + blockIdx.x] = ob;
    }
}

// Exclusive scans of the block totals (totals at iblk[2 nblk], iblk[2 nblk + 1]),
// then per destination shard its run, bases and transfer size (xrow: particles,
// rows; zero when the rule did not fire).  The shard this rank holds is planned
// too: the host picks which shard each rank keeps from these counts
// (exchange_particles), and the kept one is then skipped by the packing.
__global__ __launch_bounds__(1024) void k_pack_bounds(const ResampleParams P) {
    __shared__ long long lds[16];
    const bool fired = P.stats->resampled != 0;
    if (fired) {
        for (int half = 0; half < 2; ++half) {
            int64_t *v = P.iblk + (int64_t)half * P.nblk;
            const int per = (P.nblk + 1023) / 1024;
            const int b0 = min(P.nblk, (int)threadIdx.x * per), b1 = min(P.nblk, b0 + per);
            long long run = 0;
            for (int b = b0; b < b1; ++b) run += v[b];
            const long long incl = wave_incl_scan_i64(run);
            const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
            __syncthreads();
            if (lane == 63) lds[wid] = incl;
            __syncthreads();
            long long off = incl - run;
            for (int k = 0; k < wid; ++k) off += lds[k];
            for (int b = b0; b < b1; ++b) {
                const long long t = v[b];
                v[b] = off;
                off += t;
            }
            if (threadIdx.x == 1023) P.iblk[2 * P.nblk + half] = off;
        }
        __syncthreads();
    }
    const int p = threadIdx.x;
    if (p >= P.world) return;
    PackPlan pl{};
    if (fired) {
        const int64_t pa = shard_begin(P.N, P.world, p), pb = shard_begin(P.N, P.world, p + 1);
        plan_run(P.n, pa, pb, [&](int64_t i) { return (int64_t)P.mlo[i]; }, [&](int64_t i) { return (int64_t)P.mhi[i]; },
                 pl.i0, pl.i1);
        auto E = [&](int64_t i, int half) -> int64_t {
            return (i >= P.n) ? P.iblk[2 * P.nblk + half]
                              : P.iblk[(int64_t)half * P.nblk + i / kScanBlock] + (half ? P.rank_e[i] : P.rank_d[i]);
        };
        pl.e0 = E(pl.i0, 0);
        pl.c0 = E(pl.i0, 1);
        pl.K = E(pl.i1, 0) - pl.e0;
        pl.S = E(pl.i1, 1) - pl.c0;
        pl.pa = pa;
        pl.pb = pb;
    }
    P.plan[p] = pl;
    int64_t *xr = P.xrow + kXrowWords * p;
    xr[0] = pl.K;
    xr[1] = pl.S;
    xr[2] = 0;               // distinct pages, covariances: k_dedup_assign
    xr[3] = 0;
    xr[4] = pl.i0;
    xr[5] = pl.i1;
}

hipError_t launch_pack_count(const ResampleParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_pack_plan, dim3(p.nblk), dim3(kBlock), 0, s, p);
    hipLaunchKernelGGL(k_pack_bounds, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

// Headers of every local particle sent to another rank, into each destination's
// transfer.
__global__ __launch_bounds__(kBlock) void k_pack_headers(const ResampleParams P) {
    if (!P.stats->resampled) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= P.n) return;
    const int64_t lo = P.mlo[i], hi = P.mhi[i];
    if (lo > hi) return;
    const int64_t b = i / kScanBlock;
    const int64_t e = P.iblk[b] + P.rank_d[i], c = P.iblk[P.nblk + b] + P.rank_e[i];
    for (int p = 0; p < P.world; ++p) {
        const PackPlan &pl = P.plan[p];
        if (p == P.keep || i < pl.i0 || i >= pl.i1) continue;
        PackHeader h{};
        h.gsrc = P.a + i;
        h.out_lo = (int32_t)max(lo, pl.pa);
        h.out_hi = (int32_t)min(hi, pl.pb - 1);
        h.cnt = P.cnt[i];
        h.soff = (int32_t)(c - pl.c0);
        h.x = P.x[i];
        h.y = P.y[i];
        h.yaw = P.yaw[i];
        h.w = P.w[i];
        reinterpret_cast<PackHeader *>(P.sbuf[p])[e - pl.e0] = h;
    }
}

// ---- page dedup (XferTable) ----
__device__ __forceinline__ uint32_t xt_hash(unsigned long long key, int log2cap) {
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - log2cap));
}

// Row k of local particle i as a table key for destination p (0: the particle
// sends nothing there or has no such row).
struct DedupRow {
    unsigned long long key;
    bool single;             // the particle fills one output of p's shard
};
__device__ __forceinline__ DedupRow dedup_row(const ResampleParams &P, int p, int64_t i, int k) {
    DedupRow r{0ull, false};
    if (i < 0 || i >= P.n) return r;
    const PackPlan &pl = P.plan[p];
    if (i < pl.i0 || i >= pl.i1) return r;
    const int c = P.cnt[i];
    if (k * kPageSlots >= c) return r;
    const int64_t lo = P.mlo[i], hi = P.mhi[i];
    if (lo > hi) return r;
    const uint32_t page = *pt_entry(P.map, k, i) & kIdMask;
    const unsigned long long fill = (unsigned long long)min(kPageSlots, c - k * kPageSlots);
    r.key = (fill << 40) | ((unsigned long long)(p + 1) << 32) | page;
    r.single = max(lo, pl.pa) == min(hi, pl.pb - 1);
    return r;
}

__device__ __forceinline__ int64_t dedup_entry(const ResampleParams &P, int p, int64_t i, int k) {
    return P.xt.ebase[p] + (P.iblk[P.nblk + i / kScanBlock] + P.rank_e[i] + k - P.plan[p].c0);
}

__device__ __forceinline__ bool same_bits(double a, double b) {
    return __double_as_longlong(a) == __double_as_longlong(b);
}
// slots of a page whose covariance is not the initial one (the 8 mirror loads,
// then the records' covariance loads, issued together)
__device__ __forceinline__ uint32_t page_cov_mask(const ResampleParams &P, uint32_t page, int fill) {
    uint32_t rec[kPageSlots];
#pragma unroll
    for (int j = 0; j < kPageSlots; ++j) rec[j] = mirror_rec(load_mirror(page_ptr(P.map.pool, page), j));
    double2 b[kPageSlots], c[kPageSlots];
#pragma unroll
    for (int j = 0; j < kPageSlots; ++j) {
        const double2 *r = reinterpret_cast<const double2 *>(P.map.recs + (int64_t)rec[j < fill ? j : 0] * kRecBytes);
        b[j] = r[1];
        c[j] = r[2];
    }
    uint32_t mask = 0;
#pragma unroll
    for (int j = 0; j < kPageSlots; ++j)
        if (j < fill && !(same_bits(b[j].x, P.init_cov[0]) && same_bits(b[j].y, P.init_cov[1]) &&
                          same_bits(c[j].x, P.init_cov[2]) && same_bits(c[j].y, P.init_cov[3])))
            mask |= 1u << j;
    return mask;
}
// Every row of every particle sent: its (destination, page) key into the table,
// one thread per (particle, row) (grid y: rows; a row's descriptor loads are
// coalesced over x).  Only the first of a run of neighbours naming the same
// page inserts (siblings of one resample share every page neither has written
// since): few atomics, and the followers find the key in k_dedup_follow.  A key
// named more than once is marked shared (ref).
__global__ __launch_bounds__(kBlock) void k_dedup_insert(const ResampleParams P) {
    const int64_t i = P.xt.i_lo + (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int k = blockIdx.y;
    const XferTable &T = P.xt;
    const uint32_t mask = (uint32_t)(T.cap - 1);
    for (int p = 0; p < P.world; ++p) {
        if (p == P.keep) continue;
        const DedupRow r = dedup_row(P, p, i, k);
        if (!r.key || dedup_row(P, p, i - 1, k).key == r.key) continue;
        bool shared = dedup_row(P, p, i + 1, k).key == r.key;
        uint32_t h = xt_hash(r.key, T.log2cap);
        bool first = false;
        for (;;) {
            const unsigned long long old = atomicCAS(T.key + h, 0ull, r.key);
            if (old == 0ull) {
                first = true;
                break;
            }
            if (old == r.key) {
                shared = true;
                break;
            }
            h = (h + 1u) & mask;
        }
        if (shared) T.ref[h] = 1u;
        if (first) T.cmask[h] = page_cov_mask(P, (uint32_t)(r.key & 0xffffffffu), (int)((r.key >> 40) & 0xfu));
        T.eslot[dedup_entry(P, p, i, k)] = h | (r.single ? kEntryOwned : 0u);
    }
}

// The rows that did not insert: their key's slot (read-only probes; neighbours
// hit the same line).
__global__ __launch_bounds__(kBlock) void k_dedup_follow(const ResampleParams P) {
    const int64_t i = P.xt.i_lo + (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int k = blockIdx.y;
    const XferTable &T = P.xt;
    const uint32_t mask = (uint32_t)(T.cap - 1);
    for (int p = 0; p < P.world; ++p) {
        if (p == P.keep) continue;
        const DedupRow r = dedup_row(P, p, i, k);
        if (!r.key || dedup_row(P, p, i - 1, k).key != r.key) continue;
        uint32_t h = xt_hash(r.key, T.log2cap);
        while (T.key[h] != r.key) h = (h + 1u) & mask;
        T.eslot[dedup_entry(P, p, i, k)] = h | (r.single ? kEntryOwned : 0u);
    }
}

// Index of every distinct page among its destination's (any order: the entries
// name pages by index) and of its first covariance, the counts into
// xrow[6 p + 2] / [6 p + 3], the slot into ulist.  A workgroup takes a
// contiguous chunk of the table: it counts per destination (ballot per wave,
// LDS per workgroup), claims each destination's ranges with one global atomic
// each, then hands out indices in them.
constexpr int kAssignChunk = 16 * kBlock;
__device__ __forceinline__ void wave_dest_add(uint32_t *s_cnt, int d, uint32_t &local) {
    const int lane = threadIdx.x & 63;
    uint64_t todo = __ballot(d >= 0);
    while (todo) {
        const int lead = __builtin_ctzll(todo);
        const int dd = __shfl(d, lead, 64);
        const uint64_t m = __ballot(d == dd);
        uint32_t wb = 0;
        if (lane == lead) wb = atomicAdd(&s_cnt[dd], (uint32_t)__popcll(m));
        wb = __shfl(wb, lead, 64);
        if (d == dd) local = wb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        todo &= ~m;
    }
}
__global__ __launch_bounds__(kBlock) void k_dedup_assign(const ResampleParams P) {
    __shared__ uint32_t s_cnt[kMaxRanks], s_run[kMaxRanks], s_base[kMaxRanks];
    __shared__ uint32_t s_ccnt[kMaxRanks], s_crun[kMaxRanks], s_cbase[kMaxRanks];
    const XferTable &T = P.xt;
    const int64_t c0 = (int64_t)blockIdx.x * kAssignChunk;
    const int64_t c1 = min(c0 + kAssignChunk, T.cap);
    if (threadIdx.x < kMaxRanks) s_cnt[threadIdx.x] = s_run[threadIdx.x] = s_ccnt[threadIdx.x] = s_crun[threadIdx.x] = 0;
    __syncthreads();
    auto dest = [&](int64_t h) {
        const unsigned long long key = (h < c1) ? T.key[h] : 0ull;
        return key ? (int)((key >> 32) & 0xffu) - 1 : -1;
    };
    for (int64_t h = c0 + threadIdx.x; h < c0 + kAssignChunk; h += kBlock) {
        const int d = dest(h);
        uint32_t dummy = 0;
        wave_dest_add(s_cnt, d, dummy);
        if (d >= 0) {
            const uint32_t mask = T.cmask[h];
            if (mask) atomicAdd(&s_ccnt[d], (uint32_t)__popc(mask));
        }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)P.world) {
        unsigned long long *row = reinterpret_cast<unsigned long long *>(P.xrow + kXrowWords * threadIdx.x);
        if (s_cnt[threadIdx.x]) s_base[threadIdx.x] = (uint32_t)atomicAdd(row + 2, (unsigned long long)s_cnt[threadIdx.x]);
        if (s_ccnt[threadIdx.x])
            s_cbase[threadIdx.x] = (uint32_t)atomicAdd(row + 3, (unsigned long long)s_ccnt[threadIdx.x]);
    }
    __syncthreads();
    unsigned repeats = 0;
    for (int64_t h = c0 + threadIdx.x; h < c0 + kAssignChunk; h += kBlock) {
        const int d = dest(h);
        uint32_t local = 0;
        wave_dest_add(s_run, d, local);
        if (d >= 0) {
            const uint32_t u = s_base[d] + local;
            const uint32_t mask = T.cmask[h];
            T.uidx[h] = u;
            T.cbase[h] = mask ? s_cbase[d] + atomicAdd(&s_crun[d], (uint32_t)__popc(mask)) : 0u;
            T.ulist[T.ebase[d] + u] = (uint32_t)h;
            if (P.sent_mask) {
                // probe: did this page already go to rank d since the last collection?
                const uint32_t page = (uint32_t)T.key[h] & kIdMask, bit = 1u << d;
                repeats += (atomicOr(&P.sent_mask[page], bit) & bit) ? 1u : 0u;
            }
        }
    }
    if (P.sent_mask) {
        __shared__ unsigned long long s_rep[kBlock / 64];
        const unsigned long long r = block_sum_u64<kBlock>(repeats, s_rep);
        if (threadIdx.x == 0 && r) atomicAdd(&P.stats->repeat_pages, r);
    }
}

hipError_t launch_pack_dedup(const ResampleParams &p, hipStream_t s) {
    const unsigned g = (unsigned)((p.xt.i_hi - p.xt.i_lo + kBlock - 1) / kBlock);
    if (p.xt.i_hi > p.xt.i_lo && p.map.rows > 0) {
        hipLaunchKernelGGL(k_dedup_insert, dim3(g, (unsigned)p.map.rows), dim3(kBlock), 0, s, p);
        hipLaunchKernelGGL(k_dedup_follow, dim3(g, (unsigned)p.map.rows), dim3(kBlock), 0, s, p);
    }
    hipLaunchKernelGGL(k_dedup_assign, dim3((unsigned)((p.xt.cap + kAssignChunk - 1) / kAssignChunk)), dim3(kBlock), 0,
                       s, p);
    return hipGetLastError();
}

__device__ __forceinline__ int dest_of(const int64_t *base, int world, int64_t e) {
    int p = 0;
    while (p + 1 < world && e >= base[p + 1]) ++p;
    return p;
}

// Row entries: the page's index among the destination's distinct pages, owned
// when the particle fills one output and no other entry names the page.
__global__ __launch_bounds__(kBlock) void k_pack_index(const ResampleParams P, int64_t total) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= total) return;
    const XferTable &T = P.xt;
    const int p = dest_of(T.ebase, P.world, e);
    const uint32_t es = T.eslot[e];
    const uint32_t h = es & ~kEntryOwned;
    const bool own = (es & kEntryOwned) && T.ref[h] == 0u;
    reinterpret_cast<uint32_t *>(P.sbuf[p] + xfer_idx_off(P.plan[p].K))[e - T.ebase[p]] =
        T.uidx[h] | (own ? kEntryOwned : 0u);
}

// Distinct pages, compact (XferPage): 8 lanes per page, lane j slot j's mean,
// map index and, when it is not the initial one, covariance.
__global__ __launch_bounds__(kBlock) void k_pack_pages(const ResampleParams P, int64_t total) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t g = t / kPageSlots;
    const int j = (int)(t % kPageSlots);
    if (g >= total) return;
    const XferTable &T = P.xt;
    const int p = dest_of(T.ubase, P.world, g);
    const int64_t u = g - T.ubase[p];
    const uint32_t h = T.ulist[T.ebase[p] + u];
    const unsigned long long key = T.key[h];
    const uint32_t page = (uint32_t)(key & 0xffffffffu);
    const int fill = (int)((key >> 40) & 0xfu);
    const uint32_t mask = T.cmask[h], cb = T.cbase[h];
    const PackPlan &pl = P.plan[p];
    XferPage *xp = reinterpret_cast<XferPage *>(P.sbuf[p] + xfer_page_off(pl.K, pl.S)) + u;
    if (j == 0) {
        xp->cbase = cb;
        xp->fill = (uint8_t)fill;
        xp->cmask = (uint8_t)mask;
        xp->pad0 = 0;
        xp->pad1 = 0;
    }
    uint16_t slot = 0;
    double2 xy = make_double2(0.0, 0.0);
    if (j < fill) {
        const float4 m = load_mirror(page_ptr(P.map.pool, page), j);
        const double2 *r = reinterpret_cast<const double2 *>(P.map.recs + (int64_t)mirror_rec(m) * kRecBytes);
        slot = (uint16_t)mirror_slot(m);
        xy = r[0];
        if ((mask >> j) & 1u) {
            double2 *cv = reinterpret_cast<double2 *>(P.sbuf[p] + xfer_cov_off(pl.K, pl.S, T.ubase[p + 1] - T.ubase[p])) +
                          2 * (int64_t)(cb + (uint32_t)__popc(mask & ((1u << j) - 1u)));
            cv[0] = r[1];
            cv[1] = r[2];
        }
    }
    xp->slot[j] = slot;
    xp->xy[j] = xy;
}

hipError_t launch_pack_write(const ResampleParams &p, hipStream_t s) {
    const unsigned g = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (g) hipLaunchKernelGGL(k_pack_headers, dim3(g), dim3(kBlock), 0, s, p);
    const int64_t ne = p.xt.ebase[p.world], nu = p.xt.ubase[p.world];
    if (ne > 0) hipLaunchKernelGGL(k_pack_index, dim3((unsigned)((ne + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, p, ne);
    if (nu > 0)
        hipLaunchKernelGGL(k_pack_pages, dim3((unsigned)((nu * kPageSlots + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                           p, nu);
    return hipGetLastError();
}

__device__ __forceinline__ int peer_of(const ResampleParams &P, int k) {
    int p = 0;
    while (p + 1 < P.npeers && k >= P.peers[p + 1].kbase) ++p;
    return p;
}

// page_refs mode: every row of every particle sent, as a descriptor naming the
// page where it lives (this rank's pages get this rank's tag; a page this rank
// holds by reference keeps its owner's tag), never owned.  One thread per
// (particle, row), rows over grid y; thread (0, 0) writes each destination's
// preamble (this rank's slb and summary grid).
__global__ __launch_bounds__(kBlock) void k_pack_refs(const ResampleParams P) {
    const int64_t i = P.xt.i_lo + (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int k = blockIdx.y;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < (unsigned)P.world) {
        const int p = threadIdx.x;
        if (p != P.keep && P.plan[p].K > 0) {
            RefPreamble pre{};
            pre.slb = *P.map.slb;
            pre.org = P.map.frame.org;
            pre.cell = P.map.frame.cell;
            pre.icell = P.map.frame.icell;
            pre.rank = P.rank;
            *reinterpret_cast<RefPreamble *>(P.sbuf[p]) = pre;
        }
    }
    if (i >= P.xt.i_hi || i >= P.n) return;
    const int c = P.cnt[i];
    if (k * kPageSlots >= c || P.mlo[i] > P.mhi[i]) return;
    const Desc e = *pt_entry(P.map, k, i);
    const uint32_t t = ref_tag(e);
    XDesc d;
    d.x = ((t ? t : (uint32_t)P.rank + 1u) << kRefShift) | ref_id(e);
    // (pages carry no box: the source's workgroup row box holds this one)
    d.y = P.map.bbox ? P.map.bbox[(i / kBlock) * kBBoxRows + k] : kSumOpen;
    const int64_t c_i = P.iblk[P.nblk + i / kScanBlock] + P.rank_e[i];
    for (int p = 0; p < P.world; ++p) {
        const PackPlan &pl = P.plan[p];
        if (p == P.keep || i < pl.i0 || i >= pl.i1) continue;
        reinterpret_cast<XDesc *>(P.sbuf[p] + 64 + 64 * pl.K)[c_i - pl.c0 + k] = d;
    }
}

hipError_t launch_pack_refs(const ResampleParams &p, hipStream_t s) {
    const unsigned g = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (g) {
        // headers after each destination's preamble
        ResampleParams ph = p;
        for (int q = 0; q < p.world; ++q)
            if (ph.sbuf[q]) ph.sbuf[q] += 64;
        hipLaunchKernelGGL(k_pack_headers, dim3(g), dim3(kBlock), 0, s, ph);
    }
    const int64_t span = p.xt.i_hi - p.xt.i_lo;
    if (span > 0 && p.map.rows > 0)
        hipLaunchKernelGGL(k_pack_refs, dim3((unsigned)((span + kBlock - 1) / kBlock), (unsigned)p.map.rows),
                           dim3(kBlock), 0, s, p);
    else if (p.world > 0)
        hipLaunchKernelGGL(k_pack_refs, dim3(1, 1), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

// A box's codes on another rank's summary grid, re-coded outwards on this one's
// (the sender's bounds are exact in fp32; sum_lo / sum_hi round outwards).
__device__ __forceinline__ uint32_t recode_box(uint32_t b, const RefPreamble &pre, const SumFrame &f) {
    if (b == kSumOpen) return b;
    const SumFrame g{pre.org, pre.cell, pre.icell};
    if (g.org == f.org && g.cell == f.cell) return b;
    return sum_lo(f, sum_lo_val(g, b & 0xffu)) | (sum_hi(f, sum_hi_val(g, (b >> 8) & 0xffu)) << 8) |
           (sum_lo(f, sum_lo_val(g, (b >> 16) & 0xffu)) << 16) | (sum_hi(f, sum_hi_val(g, b >> 24)) << 24);
}

// page_refs mode: the received particles' rows (rdesc) from their tagged
// descriptors -- a page of this rank's comes home untagged (not owned), the
// boxes re-coded on this rank's grid; slb lowered to each sender's.
__global__ __launch_bounds__(kBlock) void k_unpack_refs(const ResampleParams P, int32_t nrecv) {
    const int r = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nrecv) return;
    const int q = peer_of(P, r);
    const RecvPeer &pp = P.peers[q];
    const PackHeader &h = pp.hdr[r - pp.kbase];
    const RefPreamble pre = *pp.pre;
    const int rows = (h.cnt + kPageSlots - 1) / kPageSlots;
    for (int k = lane; k < rows; k += 64) {
        XDesc d = pp.refs[h.soff + k];
        if (ref_tag(d.x) == (uint32_t)P.rank + 1u) d.x = ref_id(d.x);
        d.y = recode_box(d.y, pre, P.map.frame);
        P.rdesc[(int64_t)r * P.map.rows + k] = d;
    }
    lower_slb(P.map.slb, pre.slb);
}

// ---------------------------------------------------------------- apply ----

// the gather's page-table stores are non-temporal (A/B against plain stores: scan -3%)

// outputs filled by received particles
__global__ __launch_bounds__(kBlock) void k_scatter_recv(const ResampleParams P, int32_t nrecv) {
    if (!P.stats->resampled) return;
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= nrecv) return;
    const int p = peer_of(P, k);
    const PackHeader &h = P.peers[p].hdr[k - P.peers[p].kbase];
    for (int64_t m = h.out_lo; m <= h.out_hi; ++m) P.out_src[m - P.ao] = -(k + 1);
}

// Received distinct pages into fresh pages and records: received page u takes
// page freel[base + u], its slot j record rfreel[rbase + 8 u + j].  8 lanes per
// page (lane j: slot j) rebuild the records (the initial covariance where the
// page's mask says so) and the gate mirrors (mirror_of, the sender's own
// function of the record); the page's descriptor with its box from 8-lane
// reductions (the same box as page_box), for the output row boxes.
__global__ __launch_bounds__(kBlock) void k_unpack_pages(const ResampleParams P, int64_t nu) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t g = min(t / kPageSlots, max(nu - 1, (int64_t)0));
    const int j = (int)(t % kPageSlots);
    const bool live = t / kPageSlots < nu;
    float smin = INFINITY;           // smallest positive s received (slb)
    int q = 0;
    while (q + 1 < P.npeers && g >= P.peers[q + 1].ubase) ++q;
    const XferPage *xp = P.peers[q].pages + (g - P.peers[q].ubase);
    const int fill = xp->fill;
    const uint32_t mask = xp->cmask;
    const uint32_t id = P.alloc.freel[P.alloc.base + g];
    float bx0 = INFINITY, bx1 = -INFINITY, by0 = INFINITY, by1 = -INFINITY, bs = INFINITY;
    bool finite = true;
    if (live && j < fill) {
        const double2 xy = xp->xy[j];
        Slot sl{xy.x, xy.y, M2{P.init_cov[0], P.init_cov[1], P.init_cov[2], P.init_cov[3]}};
        if ((mask >> j) & 1u) {
            const double2 *cv = P.peers[q].covs + 2 * (int64_t)(xp->cbase + (uint32_t)__popc(mask & ((1u << j) - 1u)));
            const double2 b = cv[0], c = cv[1];
            sl.P = M2{b.x, b.y, c.x, c.y};
        }
        const uint32_t rid = P.alloc.rfreel[P.alloc.rbase + g * kPageSlots + j];
        store_rec(P.map.recs, rid, sl);
        float4 mv = with_slot(mirror_of(sl), xp->slot[j]);
        mv.w = __uint_as_float(rid);
        reinterpret_cast<float4 *>(page_ptr(P.map.pool, id))[j] = mv;
        const float s = mirror_s(mv);
        smin = s > 0.0f ? s : INFINITY;
        finite = isfinite(mv.x) && isfinite(mv.y);
        bx0 = fminf(INFINITY, mv.x);
        bx1 = fmaxf(-INFINITY, mv.x);
        by0 = fminf(INFINITY, mv.y);
        by1 = fmaxf(-INFINITY, mv.y);
        bs = fminf(INFINITY, s);
    }
#pragma unroll
    for (int o = 1; o < kPageSlots; o <<= 1) {
        bx0 = fminf(bx0, __shfl_xor(bx0, o, 64));
        bx1 = fmaxf(bx1, __shfl_xor(bx1, o, 64));
        by0 = fminf(by0, __shfl_xor(by0, o, 64));
        by1 = fmaxf(by1, __shfl_xor(by1, o, 64));
        bs = fminf(bs, __shfl_xor(bs, o, 64));
        finite = finite && (__shfl_xor((int)finite, o, 64) != 0);
    }
    if (live && j == 0) {
        XDesc d;
        d.x = id;
        if (!(finite && fill > 0) || !(bs > 0.0f))
            d.y = kSumOpen;
        else
            d.y = sum_lo(P.map.frame, bx0) | (sum_hi(P.map.frame, bx1) << 8) | (sum_lo(P.map.frame, by0) << 16) |
                  (sum_hi(P.map.frame, by1) << 24);
        P.udesc[g] = d;
    }
    lower_slb(P.map.slb, smin);
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&P.stats->new_pages, (unsigned long long)nu);
}

// Page-table rows of the received particles (rdesc [r][rows]) from their
// entries: one wave per received particle, lanes over its rows (coalesced entry
// reads and descriptor writes).
__global__ __launch_bounds__(kBlock) void k_unpack_rows(const ResampleParams P, int32_t nrecv) {
    const int r = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nrecv) return;
    const int q = peer_of(P, r);
    const RecvPeer &pp = P.peers[q];
    const PackHeader &h = pp.hdr[r - pp.kbase];
    const int rows = (h.cnt + kPageSlots - 1) / kPageSlots;
    for (int k = lane; k < rows; k += 64) {
        const uint32_t ent = pp.idx[h.soff + k];
        XDesc d = P.udesc[pp.ubase + (ent & ~kEntryOwned)];
        d.x = (d.x & kIdMask) | ((ent & kEntryOwned) ? kOwned : 0u);
        P.rdesc[(int64_t)r * P.map.rows + k] = d;
    }
}

// Outputs take their source's scalars and page-table row (fast_slam_2.py:196
// deepcopy, without copying the map: the pages are shared).  A page stays owned
// only when its source fills exactly one local output (a received row: as its
// entry says); otherwise every output copies it before its first write.
// The output workgroup's row boxes (obbox): an output's page boxes lie inside
// its source workgroup's row boxes, so the union of the row boxes of the
// workgroups its local outputs come from holds them (few: systematic resampling
// maps consecutive outputs to non-decreasing sources).  Outputs received from
// another rank have no such box: a workgroup holding some adds the unions of
// their page boxes, row by row (a wave union per row, LDS across the waves).
//
// The page-table rows of outputs with a local source are copied by the launch's
// last workgroups (gather_rows), in tiles of kTileRows (32) rows x 256 outputs taken in
// row-major order: the workgroups in flight then read and write the same few
// rows, where a lane copying its own output's every row (as the received ones
// still are, below) has each wave touch all 63 rows, 4 MB apart -- address
// translation, not bytes, held that copy at ~200 us for 252 MB at config 3.
constexpr int kTileRows = 32;        // 8 / 16 / 32 measured: profiles/r06_ab_gather_tiles.json
__device__ void gather_rows(const ResampleParams &P, int64_t wg, int64_t nwg, unsigned long long *lds_u) {
    const int64_t n = P.n;
    const int64_t nblk = (n + kBlock - 1) / kBlock;
    const int64_t tiles = (int64_t)((P.map.rows + kTileRows - 1) / kTileRows) * nblk;
    unsigned nremote = 0;            // page_refs: row entries naming another rank's page
    unsigned npages = 0;             //            of them, first sightings of a page (distinct)
    for (int64_t t = wg; t < tiles; t += nwg) {
        const int r0 = (int)(t / nblk) * kTileRows;
        const int64_t m = (t % nblk) * kBlock + threadIdx.x;
        const int32_t s = m < n ? P.out_src[m] : -1;
        if (s < 0) continue;         // (received outputs: their own rows, below)
        const int rows = (P.cnt[s] + kPageSlots - 1) / kPageSlots;
        if (r0 >= rows) continue;
        const int64_t lo = max((int64_t)P.mlo[s], P.ao), hi = min((int64_t)P.mhi[s], P.ao + n - 1);
        // (page_refs: only a source with one output in all keeps its pages -- a row
        // also sent to another rank is referenced there)
        const uint32_t keep = (P.refs ? P.mlo[s] == P.mhi[s] : hi == lo) ? 0xffffffffu : kIdMask;
        uint32_t e[kTileRows];
#pragma unroll
        for (int u = 0; u < kTileRows; ++u) e[u] = *pt_entry(P.map, min(r0 + u, rows - 1), s);
#pragma unroll
        for (int u = 0; u < kTileRows; ++u) {
            if (r0 + u < rows) {
                e[u] &= keep;
                if (P.refs && ref_tag(e[u])) {
                    ++nremote;
                    bool claimed = false;
                    if (P.tkey && ptable_insert(P.tkey, P.tcap, P.tepoch, e[u], &claimed) >= 0 && claimed)
                        ++npages;
                }
                __builtin_nontemporal_store(e[u], P.opt + (int64_t)(r0 + u) * n + m);
            }
        }
    }
    if (P.refs) {
        const unsigned long long br = block_sum_u64<kBlock>(nremote, lds_u);
        if (threadIdx.x == 0 && br) atomicAdd(&P.stats->remote_rows, br);
        __syncthreads();             // lds_u is reused below
        const unsigned long long bp = block_sum_u64<kBlock>(npages, lds_u);
        if (threadIdx.x == 0 && bp) atomicAdd(&P.stats->remote_pages, bp);
    }
}

// workgroups of launch_resample_apply's gather that copy rows (see above)
static int64_t gather_row_groups(int64_t n, int rows) {
    const int64_t tiles = (int64_t)((rows + kTileRows - 1) / kTileRows) * ((n + kBlock - 1) / kBlock);
    return std::min<int64_t>(tiles, 2048);
}

__global__ __launch_bounds__(kBlock) void k_gather_particles(const ResampleParams P) {
    __shared__ double lds_d[kBlock / 64];
    __shared__ int64_t lds_l[kBlock / 64];
    __shared__ BoxLds s_bb;
    __shared__ int s_src[kBlock];    // source workgroup of each local output (-1: none)
    __shared__ int s_sb[kBlock];     // the distinct ones, in order
    __shared__ int s_wc[kBlock / 64];
    if (P.go ? *(volatile const unsigned long long *)P.go != P.go_seq : !P.stats->resampled) return;
    __shared__ unsigned long long lds_u[kBlock / 64];
    {
        const int64_t nblk = (P.n + kBlock - 1) / kBlock;
        if ((int64_t)blockIdx.x >= nblk) {
            gather_rows(P, (int64_t)blockIdx.x - nblk, (int64_t)gridDim.x - nblk, lds_u);
            return;
        }
    }
    const int64_t m = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (m == 0 && P.runs_n) *P.runs_n = 0u;      // the runs were filled before this kernel
    const bool bb = P.obbox != nullptr && P.map.bbox != nullptr;
    if (bb) lds_box_set(s_bb, threadIdx.x, kBoxEmpty);      // kBBoxRows == kBlock
    double bv = -INFINITY;
    int64_t bi = INT64_MAX;
    unsigned slots = 0;
    const int64_t n = P.n;
    int32_t s = 0;
    int rows = 0;                    // rows of this output's map
    const XDesc *rsrc = nullptr;     // a received particle's rows (descriptors with boxes)
    if (m < n) {
        s = P.out_src[m];
        double w;
        int c;
        if (s >= 0) {
            P.ox[m] = P.x[s];
            P.oy[m] = P.y[s];
            P.oyaw[m] = P.yaw[s];
            w = P.w[s];
            c = P.cnt[s];
        } else {
            const int r = -s - 1;
            const int p = peer_of(P, r);
            const PackHeader &h = P.peers[p].hdr[r - P.peers[p].kbase];
            P.ox[m] = h.x;
            P.oy[m] = h.y;
            P.oyaw[m] = h.yaw;
            w = h.w;
            c = h.cnt;
            rsrc = P.rdesc + (int64_t)r * P.map.rows;
            rows = (c + kPageSlots - 1) / kPageSlots;     // (local outputs' rows: gather_rows)
        }
        P.ocnt[m] = c;
        P.ow[m] = w;
        bv = w;
        bi = m;
        slots = (unsigned)c;
    }
    // received outputs in this workgroup: their boxes take the row-union path below
    const bool recv = bb && __syncthreads_or(m < n && s < 0);
    if (bb) s_src[threadIdx.x] = (m < n && s >= 0) ? s / kBlock : -1;
    if (bb) __syncthreads();         // s_bb, s_src written
    // the page-table row of every received output, 8 independent loads in flight
    // per lane (one per iteration would pay a full memory latency per row); the
    // loop runs over the wave's longest such map so that every lane takes part in
    // the row unions
    const int wrows = wave_max_i(rows);
    unsigned nremote = 0;            // page_refs: row entries naming another rank's page
    unsigned npages = 0;             //            of them, first sightings of a page (distinct)
    for (int k0 = 0; k0 < wrows; k0 += 8) {
        uint32_t e[8], eb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            e[u] = 0u;
            eb[u] = kBoxEmpty;
            if (rsrc) {
                const XDesc x = rsrc[max(min(k0 + u, rows - 1), 0)];
                e[u] = x.x;
                eb[u] = x.y;
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (k0 + u < rows) {
                if (P.refs && ref_tag(e[u])) {
                    ++nremote;
                    bool claimed = false;
                    if (P.tkey && ptable_insert(P.tkey, P.tcap, P.tepoch, e[u], &claimed) >= 0 && claimed)
                        ++npages;
                }
                __builtin_nontemporal_store(e[u], P.opt + (int64_t)(k0 + u) * n + m);
            }
        }
        if (recv) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (k0 + u < wrows) {
                    const uint32_t b = wave_box_union((k0 + u < rows && s < 0) ? eb[u] : kBoxEmpty);
                    if ((threadIdx.x & 63) == 0) lds_box_merge(s_bb, k0 + u, b);
                }
            }
        }
    }
    // distinct source workgroups, compacted in output order
    int nsb = 0;
    if (bb) {
        const int t = threadIdx.x;
        const bool first = s_src[t] >= 0 && (t == 0 || s_src[t - 1] != s_src[t]);
        const uint64_t fm = __ballot(first);
        const int wid = t >> 6, lane = t & 63;
        if (lane == 0) s_wc[wid] = __popcll(fm);
        __syncthreads();
        int off = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) {
            off += (w < wid) ? s_wc[w] : 0;
            nsb += s_wc[w];
        }
        if (first) s_sb[off + __popcll(fm & ((1ull << lane) - 1ull))] = s_src[t];
    }
    if (P.refs) {
        const unsigned long long br = block_sum_u64<kBlock>(nremote, lds_u);
        if (threadIdx.x == 0 && br) atomicAdd(&P.stats->remote_rows, br);
        __syncthreads();             // lds_u is reused below
        const unsigned long long bp = block_sum_u64<kBlock>(npages, lds_u);
        if (threadIdx.x == 0 && bp) atomicAdd(&P.stats->remote_pages, bp);
        __syncthreads();
    }
    // per-block partials (no same-address atomics), folded by estimate_body
    const unsigned long long bs = block_sum_u64<kBlock>(slots, lds_u);
    block_argmax<kBlock>(bv, bi, lds_d, lds_l);
    if (threadIdx.x == 0) {
        P.part_best_w[blockIdx.x] = bv;
        P.part_best_i[blockIdx.x] = bi;
        P.part_slots[blockIdx.x] = bs;
    }
    // (the barriers above order every LDS write before these reads)
    if (bb && (int)threadIdx.x < P.map.rows) {
        uint32_t b = lds_box_get(s_bb, threadIdx.x);
        for (int q = 0; q < nsb; ++q) b = box_union(b, P.map.bbox[(int64_t)s_sb[q] * kBBoxRows + threadIdx.x]);
        P.obbox[(int64_t)blockIdx.x * kBBoxRows + threadIdx.x] = b;
    }
}

// Workgroup row boxes of every map from its pages' mirrors (after imports, or
// when the summary grid changes): per row, the wave union of its lanes' page
// boxes, merged across the waves in LDS.
__global__ __launch_bounds__(kBlock) void k_bbox_build(const MapRef map, const int32_t *cnt, int64_t n) {
    __shared__ BoxLds s_bb;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    lds_box_set(s_bb, threadIdx.x, kBoxEmpty);
    const int c = (i < n) ? cnt[i] : 0;
    const int rows = (c + kPageSlots - 1) / kPageSlots;
    __syncthreads();
    const int wrows = wave_max_i(rows);
    for (int r = 0; r < wrows; ++r) {
        uint32_t b = kBoxEmpty;
        if (r < rows) {
            // (page_refs: the page may live on another rank)
            const float4 *mir = reinterpret_cast<const float4 *>(page_ptr_any(map, *pt_entry(map, r, i)));
            b = page_box(mir, min(kPageSlots, c - r * kPageSlots), map.frame);
        }
        b = wave_box_union(b);
        if ((threadIdx.x & 63) == 0) lds_box_merge(s_bb, r, b);
    }
    __syncthreads();
    if ((int)threadIdx.x < map.rows) map.bbox[(int64_t)blockIdx.x * kBBoxRows + threadIdx.x] = lds_box_get(s_bb, threadIdx.x);
}

hipError_t launch_bbox_build(MapRef map, const int32_t *cnt, hipStream_t s) {
    if (!map.bbox) return hipSuccess;
    const unsigned g = (unsigned)((map.n + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_bbox_build, dim3(g), dim3(kBlock), 0, s, map, cnt, map.n);
    return hipGetLastError();
}

// this rank's first maximum over its outputs -> record (post-resample estimate);
// the gather's slot partials -> resample_slots
__device__ void estimate_body(const ResampleParams &P, int32_t nparts) {
    __shared__ double lds_d[16];
    __shared__ int64_t lds_l[16];
    __shared__ unsigned long long lds_u[16];
    double bv = -INFINITY;
    int64_t bi = INT64_MAX;
    unsigned long long sl = 0;
    for (int k = threadIdx.x; k < nparts; k += 1024) {
        argmax_combine(bv, bi, P.part_best_w[k], P.part_best_i[k]);
        sl += P.part_slots[k];
    }
    block_argmax<1024>(bv, bi, lds_d, lds_l);
    sl = block_sum_u64<1024>(sl, lds_u);
    if (threadIdx.x == 0) {
        P.stats->resample_slots = sl;
        RankRecord r = *P.rec;
        r.best_w = bv;
        // (before the gather the key is k_ranges': output << 32 | its source)
        const int64_t bo = (P.est_early && bi != INT64_MAX) ? (bi >> 32) : bi;
        r.best_gidx = (bo == INT64_MAX) ? INT64_MAX : P.ao + bo;
        if (bo != INT64_MAX) {
            if (P.est_early) {          // before the gather: the output's source (k_ranges)
                const int32_t s = (int32_t)(bi & 0xffffffffll);
                r.pose[0] = P.x[s];
                r.pose[1] = P.y[s];
                r.pose[2] = P.yaw[s];
            } else {
                r.pose[0] = P.ox[bo];
                r.pose[1] = P.oy[bo];
                r.pose[2] = P.oyaw[bo];
            }
        }
        *P.rec = r;
    }
}

__global__ __launch_bounds__(1024) void k_estimate(const ResampleParams P, int32_t nparts) {
    if (P.stats->resampled) estimate_body(P, nparts);
}

// One GPU, end of a scan that resampled: the estimate after the resample and
// the stats publication (k_estimate + k_global_best + k_publish in one launch);
// a scan without a resample was published by k_finalize (stats zeroed).
__global__ __launch_bounds__(1024) void k_tail_single(const ResampleParams R, const ReduceParams P, int32_t nparts,
                                                     DevStats *host_stats, unsigned long long *host_flag,
                                                     unsigned long long seq) {
    if (!R.stats->resampled) return;
    if (blockIdx.x > 0) {                  // the other workgroups: k_ranges' listed runs
        fill_runs_body(R, blockIdx.x - 1, gridDim.x - 1);
        return;
    }
    estimate_body(R, nparts);
    __syncthreads();
    if (threadIdx.x == 0) {
        global_best_body(P);
        if (R.gen) *R.gen += 1u;        // the other set is current (BufSet; the next kernels read it)
        if (R.go) *R.go = R.go_seq;     // (published before the gather: it runs on this marker)
    }
    __syncthreads();
    publish_body(P.stats, host_stats, host_flag, seq);
}

hipError_t launch_tail_single(const ResampleParams &r, const ReduceParams &p, DevStats *host_stats,
                              unsigned long long *host_flag, unsigned long long seq, hipStream_t s,
                              hipEvent_t e1) {
    const int32_t nparts = (int32_t)((r.n + kBlock - 1) / kBlock);
    // one workgroup for the tail, kTailFill more for the runs k_ranges listed (none
    // listed: they return at once -- cheaper than a kernel of their own every scan)
    const unsigned fill = ((r.ranges_mode & 2) && r.runs) ? kTailFill : 0u;
    FS2_LAUNCH_EV(k_tail_single, dim3(1 + fill), dim3(1024), s, nullptr, e1, r, p, nparts, host_stats, host_flag, seq);
    return hipGetLastError();
}

hipError_t launch_resample_apply(const ResampleParams &p, bool estimate, hipStream_t s) {
    const unsigned g = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (g == 0) return hipSuccess;
    int32_t nrecv = 0;
    int64_t nu = 0;
    for (int q = 0; q < p.npeers; ++q) {
        nrecv += p.peers[q].K;
        nu += p.peers[q].U;
    }
    if (nrecv > 0) {
        hipLaunchKernelGGL(k_scatter_recv, dim3((nrecv + kBlock - 1) / kBlock), dim3(kBlock), 0, s, p, nrecv);
        if (p.refs) {
            hipLaunchKernelGGL(k_unpack_refs, dim3((nrecv + kBlock / 64 - 1) / (kBlock / 64)), dim3(kBlock), 0, s, p,
                               nrecv);
        } else {
            if (nu > 0)
                hipLaunchKernelGGL(k_unpack_pages, dim3((unsigned)((nu * kPageSlots + kBlock - 1) / kBlock)),
                                   dim3(kBlock), 0, s, p, nu);
            hipLaunchKernelGGL(k_unpack_rows, dim3((nrecv + kBlock / 64 - 1) / (kBlock / 64)), dim3(kBlock), 0, s, p,
                               nrecv);
        }
    }
    // (the per-output blocks first, then the row tiles: gather_rows)
    hipLaunchKernelGGL(k_gather_particles, dim3(g + (unsigned)gather_row_groups(p.n, p.map.rows)), dim3(kBlock), 0,
                       s, p);
    if (estimate) hipLaunchKernelGGL(k_estimate, dim3(1), dim3(1024), 0, s, p, (int32_t)g);
    return hipGetLastError();
}

}  // namespace fs2
