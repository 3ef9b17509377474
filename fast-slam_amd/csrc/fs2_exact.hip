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
// term, or the chain's first element are evaluated in order from their exact
// entry value (chain_unit, fs2_chain.hpp).  Only those (~20-40 per chain: one
// per binade crossed) are walked serially; the translations between them are an
// integer scan.  A term below half the step of its estimate's lower binade adds
// 0 wherever the chain is; a unit of such terms alone is a translation by 0 even
// when the estimate straddles a binade boundary, its binade inherited from the
// last translation unit before it (chain_elast: a run's binade is constant, and a
// run of identities alone adds nothing) -- a collapsed resample's million tiny
// weights after a chain ending within the margin of 2^0 are one scan, not a walk.
//
//   k_chain_units  per unit: translation (binade E, D) or serial (each workgroup
//                  estimates the chain at its block starts from the block sums
//                  before it; in total mode 8 more workgroups fold the update
//                  pass's counters, k_wsum's other job)
//   k_chain_walk   one workgroup: integer scan of D, then the serial units in
//                  order (wave 0; chain_unit evaluates a unit in a few wave-wide
//                  steps: one per binade crossed or tie, not one per term)
// In prefix mode the resample's range kernel evaluates the translation units'
// values itself (s_in + (scan of rint(a / u)) u, fs2_chain.hpp), so the running
// sum is never materialised beyond the serial units.
//
// numpy sum of squares.  Each full 8192-element chunk is numpy's pairwise tree:
// 64 leaves of 128 elements (8 accumulators of 16 sequential adds, combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))), the leaves combined as a balanced
// binary tree in order.  k_normalize sums the leaves of its 256 weights as it
// writes them; k_finalize adds each chunk's leaves up the tree (one wave per
// chunk, xor butterflies), sums a partial last chunk with numpy's recursion
// (np_pairwise_partial, fs2_chain.hpp) and adds the chunk sums in order.
#include "fs2_chain.hpp"

namespace fs2 {

__device__ __forceinline__ bool lazy_skip(const ChainParams &P) {
    return P.stats != nullptr && !P.stats->resampled;
}

// --------------------------------------------------------------- chain ----

// Per 64-term unit (one wave; kChainGroup units per 1024-thread workgroup).
// Each term's chain value before and after it is estimated (block prefix + wave
// scan) with the margin; a term is "translation" in binade E when both bounds
// lie in E, it is finite, >= 0, not a tie and not the chain's first term.  A
// unit whose terms all translate in one binade is one translation D (uinfo,
// udelta); otherwise ("listed") its runs of translating terms with equal E and
// its other terms (one each) become up to kChainSegs segments (urec; a unit
// with more is evaluated term by term by chain_unit in the walk).  The
// workgroup also scans its units: ugl / uol (exclusive D, inclusive listed
// count inside the group) and the group's totals bD / bC / bM (listed mask).
__global__ __launch_bounds__(1024) void k_chain_units(const ChainParams P) {
    __shared__ double s_ws[16];
    __shared__ unsigned long long s_D[16];
    __shared__ int s_f[16], s_e[16];
    __shared__ double s_red[16], s_bp[4];
    __shared__ unsigned long long s_c[16][kNumCounters];
    if (P.lazy && lazy_skip(P)) return;
    FS2_TS_DECL;
    FS2_TS(0, 0);
    const int64_t ngroups = (P.n + 1023) / 1024;
    if (blockIdx.x >= ngroups) {     // the update pass's counters (total mode)
        fold_counters(P.cpart, P.ncpart, P.cstats, (int)(blockIdx.x - ngroups), s_c);
        return;
    }
    // this thread's term, requested before the block-prefix loads below (one memory
    // latency for both)
    const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    const bool valid = i < P.n;
    const double a = valid ? P.a[i] : 0.0;
    {
        // estimates of the chain at this workgroup's four 256-term block starts:
        // the block sums before them in any order (the margin bounds every order).
        // Every load is issued before any add (four per thread and round), and the
        // workgroup's own four block sums come with them: one memory latency, not
        // one per loop step.
        const int64_t nb0 = (int64_t)blockIdx.x * 4;
        const int t = threadIdx.x;
        const double own = (t < 4 && nb0 + t < P.nb) ? P.bsum[nb0 + t] : 0.0;
        double v = 0.0;
        for (int64_t j0 = 0; j0 < nb0; j0 += 4096) {
            double x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t j = j0 + t + 1024 * u;
                x[u] = (j < nb0) ? P.bsum[j] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) v += x[u];
        }
        // (sharded: plus the tree prefix of the shards before this one)
        const double base = block_sum<1024>(v, s_red) + (P.est_base ? *P.est_base : 0.0);
        if (t < 64) {
            const double b0 = bcast(own, 0), b1 = bcast(own, 1), b2 = bcast(own, 2);
            if (t < 4) {
                double e = base;
                if (t > 0) e += b0;
                if (t > 1) e += b1;
                if (t > 2) e += b2;
                s_bp[t] = e;
            }
        }
        __syncthreads();
    }
    FS2_TS(0, 1);
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int64_t k = (int64_t)blockIdx.x * kChainGroup + wid;
    const int64_t nu = (P.n + kUnit - 1) / kUnit;
    const double incl = wave_incl_scan_f64(a);
    if (lane == 63) s_ws[wid] = incl;
    __syncthreads();
    unsigned long long D = 0;
    int listed = 0, etr = 0;                         // etr: binade + 4096 of a translation proper
    if (k < nu) {
        // estimate of the chain before this unit: the 256-term block prefix, then
        // the units of that block ahead of this one
        const int c4 = wid >> 2;
        double e_in = s_bp[c4];
        for (int q = 4 * c4; q < wid; ++q) e_in += s_ws[q];
        const double lo = (e_in + (incl - a)) * (1.0 - P.margin), hi = (e_in + incl) * (1.0 + P.margin);
        // [0, 2^-1021) -- zero, the subnormals and the lowest normal binade -- is one
        // grid of step 2^-1074 (binade -1022 below): every add there is exact, so a
        // run of zero or subnormal weights (a diverged filter's underflowed
        // likelihoods) is a translation too, not a unit walked term by term
        const bool base = valid && !(i == 0 && P.chain_first) && a >= 0.0 && a < INFINITY && lo >= 0.0 &&
                          hi < 0x1p1020;
        const int E = base ? chain_binade(lo) : -4096;
        bool ok = base && chain_binade(hi) == E;
        // A term below half the step of binade E leaves the chain where it is in E and
        // in every binade above (round to nearest, no tie): an exact identity wherever
        // in [lo, hi] the chain is, even when that estimate straddles a binade
        // boundary.  Without this a long run of tiny weights after a chain that ends
        // within the estimate's margin of a power of two (a resample whose normalised
        // weights sum to 1 - 6e-11: 2600 units, 2.5 ms in k_chain_walk) was walked
        // term by term; a unit of identities alone is a translation by 0 whose binade
        // is inherited (chain_elast), one that mixes them with other terms is listed.
        const bool ident = base && !ok && scaled(a, E) < 0.5;
        long long r = 0;
        if (ok) {
            const double q = scaled(a, E);          // < 2^53: exact
            ok = q - floor(q) != 0.5;               // a tie: the rounding depends on s
            r = ok ? (long long)rint(q) : 0;
        }
        const bool okt = ok;                        // a translation term proper (in binade E)
        ok = ok || ident;                           // segments may also hold identities (r = 0)
        const unsigned long long vmask = __ballot(valid);
        const int E0 = __builtin_amdgcn_readfirstlane(E);
        if (k == 0 && P.chain_first) {
            // the chain's first unit: its entry is known, so its values are evaluated
            // here; the walk only sets the value after it
            listed = 1;
            double s0 = 0.0;
            const double mine = chain_unit(a, __popcll(vmask), s0, true);
            if (P.c && valid) P.c[i] = mine;
            if (lane == 0) {
                UnitRec rec;
#pragma unroll
                for (int g = 0; g < kChainSegs; ++g) {
                    rec.meta[g] = 0;
                    rec.val[g] = 0.0;
                }
                rec.meta[0] = __popcll(vmask) | 0x80;
                rec.val[0] = s0;                     // the value after the unit (set, not added)
                P.uinfo[k] = 1 | (1 << 3);
                P.udelta[k] = 0;
                P.urec[k] = rec;
            }
        } else if (!(k == 0 && P.force_list0) && __ballot(okt && E == E0) == vmask) {    // one translation
            // (a sharded rank lists its unit 0: the walk and the ranges need a listed
            // unit before every translation, and the chain enters there from another rank)
            D = (unsigned long long)wave_sum_i64(r);
            etr = E0 + 4096;
            if (lane == 0) {
                P.uinfo[k] = (E0 + 4096) << 2;
                P.udelta[k] = (long long)D;
            }
        } else if (!(k == 0 && P.force_list0) && __ballot(ok && r == 0) == vmask) {   // identities only
            if (lane == 0) {
                P.uinfo[k] = ((E0 + 4096) << 2) | 2;
                P.udelta[k] = 0;
            }
        } else {
            listed = 1;
            const int okp = __shfl_up(ok ? 1 : 0, 1, 64), Ep = __shfl_up(E, 1, 64);
            const bool start = valid && (lane == 0 || !ok || !okp || E != Ep);
            unsigned long long sm = __ballot(start);
            const unsigned long long okm = __ballot(ok);
            const int nseg = __popcll(sm);
            if (nseg > kChainSegs) {
                if (lane == 0) {
                    P.uinfo[k] = 3;
                    P.udelta[k] = 0;
                }
            } else {
                const long long ir = wave_incl_scan_i64(r);
                const int cnt = __popcll(vmask);
                UnitRec rec;
#pragma unroll
                for (int g = 0; g < kChainSegs; ++g) {
                    rec.meta[g] = 0;
                    rec.val[g] = 0.0;
                    if (sm) {
                        const int st = (int)__builtin_ctzll(sm);
                        sm &= sm - 1;
                        const int en = sm ? (int)__builtin_ctzll(sm) : cnt;
                        if ((okm >> st) & 1ull) {
                            const int Es = __builtin_amdgcn_readlane(E, st);
                            rec.meta[g] = (en - st) | ((Es + 4096) << 8);
                            const long long Dg = bcast_i64(ir, en - 1) - (st > 0 ? bcast_i64(ir, st - 1) : 0ll);
                            rec.val[g] = (double)Dg * unit_ulp(Es);   // exact: D < 2^53
                        } else {
                            rec.meta[g] = 1 | 0x80;
                            rec.val[g] = bcast(a, st);
                        }
                    }
                }
                if (lane == 0) {
                    P.uinfo[k] = 1 | (nseg << 3);
                    P.udelta[k] = 0;
                    P.urec[k] = rec;
                }
            }
        }
    }
    FS2_TS(0, 2);
    if (lane == 0) {
        s_D[wid] = D;
        s_f[wid] = listed;
        s_e[wid] = etr;
    }
    __syncthreads();
    if (t < kChainGroup) {
        // the group's scan (16 values, lanes 0..15 of wave 0)
        unsigned long long dx = 0;
        int cx = 0, ex = 0;
        unsigned mask = 0;
        for (int q = 0; q < kChainGroup; ++q) {
            if (q < t) dx += s_D[q];
            if (q <= t) cx += s_f[q];
            if (q <= t && s_e[q]) ex = s_e[q];
            mask |= (unsigned)s_f[q] << q;
        }
        const int64_t kk = (int64_t)blockIdx.x * kChainGroup + t;
        if (kk < nu) {
            P.ugl[kk] = dx;
            P.uol[kk] = cx;
            P.uel[kk] = ex;
        }
        if (t == kChainGroup - 1) {
            P.bD[blockIdx.x] = dx + s_D[t];
            P.bC[blockIdx.x] = cx;
            P.bM[blockIdx.x] = mask;
            P.bE[blockIdx.x] = ex;
        }
    }
    FS2_TS(0, 3);
}

__device__ __forceinline__ int seg_len(int32_t m) { return m & 0x7f; }
__device__ __forceinline__ bool seg_serial(int32_t m) { return (m & 0x80) != 0; }
__device__ __forceinline__ int seg_binade(int32_t m) { return (m >> 8) - 4096; }

__device__ __forceinline__ int unit_nseg(int32_t info) { return (info >> 3) & 15; }

// One workgroup.  (1) The scan over the groups' totals (k_chain_units), one
// group per thread: bpd / bpc (exclusive translation sum and listed count
// before each group) and the list of listed units in order.  (2) Wave 0 walks those in order,
// 64 at a time (their table entries and segments loaded at once, one unit per
// lane, then read lane by lane): the translation run before each is one exact
// add, a segmented unit one add per segment, a unit of many segments
// chain_unit.  Writes sentry / sout (the value before / after each), the
// total, and in prefix mode (3) every value inside the non-translation units
// (all waves, one unit each).
constexpr int kWalkStage = 32;          // term-by-term units staged in LDS per batch

// Optional phase timing of k_chain_walk (build with -DFS2_PHASE_TIMING; read back
// with fs2_debug_chain_times): summed s_memtime cycles of wave 0 per phase, calls,
// units walked, units evaluated term by term.
#ifdef FS2_PHASE_TIMING
__device__ unsigned long long g_chain[8];
#define FS2_CHAIN_STAMP(k)                                                              \
    do {                                                                                \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                     \
        if (t == 0 && (k) > 0) atomicAdd(&g_chain[(k) - 1], t_ - ch_last);              \
        ch_last = t_;                                                                   \
    } while (0)
#else
#define FS2_CHAIN_STAMP(k) do { } while (0)
#endif

// Sharded ranks: this shard's chain as a list of fp64 adds (ChainSummary), exact
// for its true entry value: per listed unit (in order) the translation run before
// it (one add of D ulp(E), exact inside binade E) and its own adds -- one per
// segment, or every term of a unit evaluated term by term (and of the chain's
// first unit: 0 + a_0 = a_0, Python's sum starting from 0); then the run after the
// last one.  Wave 0; each listed unit's first op index into P.uop.
__device__ void chain_export(const ChainParams &P, int nseq, int64_t nu, unsigned long long dtot) {
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    ChainSummary *S = P.ops_out;
    int base = 0;
    unsigned long long gprev = 0;
    for (int o0 = 0; o0 < nseq; o0 += 64) {
        const int ol = o0 + lane;
        const bool in = ol < nseq;
        int64_t q = 0;
        int32_t info = 0;
        unsigned long long g = 0;
        int Eb = 0;                                   // the binade of the run before q
        if (in) {
            q = P.seql[ol];
            info = P.uinfo[q];
            g = P.bpd[q / kChainGroup] + P.ugl[q];
            if (q > 0) Eb = chain_elast(P.uel, P.bpe, q - 1);
        }
        const unsigned long long gp = __shfl_up(g, 1, 64);
        const unsigned long long gb = (lane == 0) ? gprev : gp;
        const double run = (in && ol > 0) ? (double)(long long)(g - gb) * unit_ulp(Eb) : 0.0;
        const int cnt = in ? (int)min<int64_t>(kUnit, P.n - q * kUnit) : 0;
        const bool terms = in && ((info & 2) || (q == 0 && P.chain_first));
        const int nrun = (run != 0.0) ? 1 : 0;
        const int nops = in ? nrun + (terms ? cnt : unit_nseg(info)) : 0;
        const long long incl = wave_incl_scan_i64(nops);
        const int off = base + (int)(incl - nops);
        if (in) {
            P.uop[ol] = off + nrun;
            int k = off;
            if (nrun) {
                if (k < kChainOpsCap) S->ops[k] = run;
                ++k;
            }
            if (!terms) {
                const UnitRec rr = P.urec[q];
                const int ns = unit_nseg(info);
#pragma unroll
                for (int u = 0; u < kChainSegs; ++u)
                    if (u < ns && k + u < kChainOpsCap) S->ops[k + u] = rr.val[u];
            }
        }
        // the terms of units evaluated term by term: the wave copies them unit by unit
        for (unsigned long long tm = __ballot(terms); tm; tm &= tm - 1) {
            const int j = (int)__builtin_ctzll(tm);
            const int64_t qj = (int64_t)__builtin_amdgcn_readlane((int)q, j);
            const int oj = __builtin_amdgcn_readlane(off + nrun, j), cj = __builtin_amdgcn_readlane(cnt, j);
            if (lane < cj && oj + lane < kChainOpsCap) S->ops[oj + lane] = P.a[qj * kUnit + lane];
        }
        const int nb = min(64, nseq - o0);
        base += (int)bcast_i64(incl, 63);
        gprev = bcast_i64((long long)g, nb - 1);
    }
    if (lane == 0) {
        int k = base;
        const double run = (double)(long long)(dtot - gprev) * unit_ulp(chain_elast(P.uel, P.bpe, nu - 1));
        if (run != 0.0) {
            if (k < kChainOpsCap) S->ops[k] = run;
            ++k;
        }
        S->nops = k;
    }
}

__global__ __launch_bounds__(1024) void k_chain_walk(const ChainParams P) {
    __shared__ unsigned long long s_d[2][16];
    __shared__ int s_c[2][16], s_e[2][16];
    __shared__ int s_nseq;
    __shared__ unsigned long long s_dtot;
    __shared__ double s_terms[kWalkStage][kUnit];     // term-by-term units of a batch: terms, then values
    if (P.lazy && lazy_skip(P)) return;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
#ifdef FS2_PHASE_TIMING
    unsigned long long ch_last = 0;
#endif
    FS2_CHAIN_STAMP(0);
    const int64_t nu = (P.n + kUnit - 1) / kUnit;
    if (nu == 0) {
        if (t == 0 && P.total) *P.total = 0.0;
        return;
    }
    // (1) the scan over groups of kChainGroup units (one group per thread and step)
    const int64_t ng = (nu + kChainGroup - 1) / kChainGroup;
    unsigned long long carry = 0;
    int ccount = 0, ecarry = 0;
    for (int64_t j0 = 0; j0 < ng; j0 += 1024) {
        const int64_t gi = j0 + t;
        const bool in = gi < ng;
        const unsigned long long d = in ? P.bD[gi] : 0ull;
        const int f = in ? P.bC[gi] : 0;
        const unsigned m = in ? P.bM[gi] : 0u;
        const int e = in ? P.bE[gi] : 0;
        const int b = (int)((j0 >> 10) & 1);
        unsigned long long di = d;
        int ci = f, ei = e;                       // ei: the last nonzero binade up to this group
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long v = __shfl_up(di, o, 64);
            const int c = __shfl_up(ci, o, 64);
            const int x = __shfl_up(ei, o, 64);
            if (lane >= o) {
                di += v;
                ci += c;
                if (!ei) ei = x;
            }
        }
        const int eb = __shfl_up(ei, 1, 64);     // up to the group before (lane > 0)
        if (lane == 63) {
            s_d[b][wid] = di;
            s_c[b][wid] = ci;
            s_e[b][wid] = ei;
        }
        __syncthreads();                          // s_d[b] is rewritten two steps later
        unsigned long long dx = carry + di - d, tot = 0;
        int cx = ccount + ci - f, ctot = 0, ex = ecarry;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if (q < wid) {
                dx += s_d[b][q];
                cx += s_c[b][q];
                if (s_e[b][q]) ex = s_e[b][q];
            }
            tot += s_d[b][q];
            ctot += s_c[b][q];
            if (s_e[b][q]) ecarry = s_e[b][q];
        }
        if (lane > 0 && eb) ex = eb;
        if (in) {
            P.bpd[gi] = dx;
            P.bpc[gi] = cx;
            P.bpe[gi] = ex;
            for (unsigned mm = m; mm; mm &= mm - 1) P.seql[cx++] = (int32_t)(gi * kChainGroup + __builtin_ctz(mm));
        }
        carry += tot;
        ccount += ctot;
    }
    if (t == 0) {
        s_nseq = ccount;
        s_dtot = carry;
    }
    __syncthreads();
    const int nseq = s_nseq;
    FS2_CHAIN_STAMP(1);
    if (P.ops_out) {                 // sharded: export this shard's ops instead of walking
        chain_export(P, nseq, nu, s_dtot);
        return;
    }
#ifdef FS2_PHASE_TIMING
    if (t == 0) {
        atomicAdd(&g_chain[4], 1ull);
        atomicAdd(&g_chain[5], (unsigned long long)nseq);
    }
#endif
    // (2) 64 listed units at a time: every wave loads their table entries (one
    // per lane); the term-by-term ones have their terms staged in LDS by all
    // waves; wave 0 walks; then the staged values are written out
    double s = P.s_entry ? *P.s_entry : 0.0;       // the running value (wave 0)
    // the binade of the run after the last listed unit, requested now (read at the end)
    const int e_end = (t == 0 && P.total) ? chain_elast(P.uel, P.bpe, nu - 1) : 0;
    unsigned long long gprev = 0;
    for (int o0 = 0; o0 < nseq; o0 += 64) {
        const int ol = o0 + lane;
        int64_t q = 0;
        unsigned long long g = 0;
        int32_t info = 0, Eb = 0;                    // Eb: the binade of the run before q
        if (ol < nseq) {
            q = P.seql[ol];
            info = P.uinfo[q];
            if (wid == 0) {
                g = P.bpd[q / kChainGroup] + P.ugl[q];
                if (q > 0) Eb = chain_elast(P.uel, P.bpe, q - 1);
            }
        }
        const unsigned long long wsm = __ballot(ol < nseq && (info & 2));   // term by term
        const int nb = min(64, nseq - o0);
        // stage the term-by-term units' terms (the j-th of them into slot j % kWalkStage)
        {
            unsigned long long m = wsm;
            for (int r = 0; m; ++r) {
                const int j = (int)__builtin_ctzll(m);
                m &= m - 1;
                if (r % 16 != wid || r >= kWalkStage) continue;
                const int64_t qj = (int64_t)__builtin_amdgcn_readlane((int)q, j);
                const int64_t i = qj * kUnit + lane;
                s_terms[r][lane] = (i < P.n) ? P.a[i] : 0.0;
            }
        }
        __syncthreads();
        if (wid == 0) {
            // the batch's table in registers, one unit per lane: its segment values
            // and the exact translation run ahead of it (from the previous listed
            // unit's table entries, one lane back; the batch before for lane 0).  The
            // serial walk below reads them with readlane (scalar operands of the
            // adds), not through LDS: one dependent fp64 add per step.
            double rv[kChainSegs];
#pragma unroll
            for (int u = 0; u < kChainSegs; ++u) rv[u] = 0.0;
            if (ol < nseq && !(info & 2)) {
                const UnitRec rr = P.urec[q];
#pragma unroll
                for (int u = 0; u < kChainSegs; ++u) rv[u] = rr.val[u];
            }
            const unsigned long long gp = __shfl_up(g, 1, 64);
            const unsigned long long gb = (lane == 0) ? gprev : gp;
            const double run = (ol > 0 && ol < nseq) ? (double)(long long)(g - gb) * unit_ulp(Eb) : 0.0;
            gprev = bcast_i64((long long)g, nb - 1);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            FS2_CHAIN_STAMP(2);
            double my_entry = 0.0, my_out = 0.0;      // lane j keeps unit o0 + j's values
            int r = 0;                                // term-by-term units seen
            for (int j = 0; j < nb; ++j) {
                const int32_t infoj = __builtin_amdgcn_readlane(info, j);
                s = s + bcast(run, j);                // the translation run between (exact)
                if (lane == j) my_entry = s;
                if (infoj & 2) {
                    const int64_t qj = (int64_t)__builtin_amdgcn_readlane((int)q, j);
#ifdef FS2_PHASE_TIMING
                    if (t == 0) atomicAdd(&g_chain[6], 1ull);
#endif
                    const int cnt = (int)min<int64_t>(kUnit, P.n - qj * kUnit);
                    if (r < kWalkStage) {
                        const double mine = chain_unit(s_terms[r][lane], cnt, s, qj == 0 && P.chain_first);
                        s_terms[r][lane] = mine;
                    } else {                          // beyond the stage: from memory
                        const int64_t i = qj * kUnit + lane;
                        const double a = (i < P.n) ? P.a[i] : 0.0;
                        const double e = s;
                        const double mine = chain_unit(a, cnt, s, qj == 0 && P.chain_first);
                        if (P.c && lane < cnt) P.c[i] = mine;
                        if (P.c && qj > 0 && lane == 0) P.c[qj * kUnit - 1] = e;
                    }
                    ++r;
                } else {
                    // one add per segment (unit 0: the value after it, set)
                    const int ns = unit_nseg(infoj);
                    if (__builtin_amdgcn_readlane((int)q, j) == 0 && P.chain_first) s = bcast(rv[0], j);
                    else {
#pragma unroll
                        for (int u = 0; u < kChainSegs; ++u)
                            if (u < ns) s = s + bcast(rv[u], j);
                    }
                }
                if (lane == j) my_out = s;
            }
            if (lane < nb) {
                P.sentry[o0 + lane] = my_entry;
                P.sout[o0 + lane] = my_out;
            }
        }
        if (!wsm && o0 + 64 >= nseq) break;      // nothing staged, no further batch
        __syncthreads();
        if (P.c) {
            // the staged term-by-term units' values, and the value before each
            unsigned long long m = wsm;
            for (int r = 0; m; ++r) {
                const int j = (int)__builtin_ctzll(m);
                m &= m - 1;
                if (r % 16 != wid || r >= kWalkStage) continue;
                const int64_t qj = (int64_t)__builtin_amdgcn_readlane((int)q, j);
                const int64_t i = qj * kUnit + lane;
                if (i < P.n) P.c[i] = s_terms[r][lane];
                if (qj > 0 && lane == 0) P.c[qj * kUnit - 1] = P.sentry[o0 + j];
            }
        }
        __syncthreads();
    }
    FS2_CHAIN_STAMP(3);
    if (wid == 0 && lane == 0 && P.total) {
        // the chain ends in the translation run after the last listed unit (if any)
        *P.total = s + (double)(long long)(s_dtot - gprev) * unit_ulp(e_end);
    }
    if (!P.c) return;
    __syncthreads();                             // sentry of the last batch
    // (3) prefix mode: the values inside the segmented units, one unit per wave
#ifdef FS2_AB_NO_PHASE3
    if (true) return;                 // (timing probe only)
#endif
    for (int o = wid; o < nseq; o += 16) {
        const int64_t q = P.seql[o];
        const int32_t info = P.uinfo[q];
        if ((info & 2) || (q == 0 && P.chain_first)) continue;   // written above / by k_chain_units
        const UnitRec r = P.urec[q];
        double sg = P.sentry[o];
        const int cnt = (int)min<int64_t>(kUnit, P.n - q * kUnit);
        const int64_t i = q * kUnit + lane;
        const double a = (i < P.n) ? P.a[i] : 0.0;
        if (q > 0 && lane == 0) P.c[q * kUnit - 1] = sg;
        double mine = 0.0;
        int st = 0;
#pragma unroll
        for (int g = 0; g < kChainSegs; ++g) {
            const int32_t m = r.meta[g];
            const int len = seg_len(m);
            if (len == 0) break;
            const bool in = lane >= st && lane < st + len;
            if (seg_serial(m)) {
                if (in) mine = sg + a;
                sg = sg + r.val[g];
            } else {
                const int E = seg_binade(m);
                const double u = unit_ulp(E);
                const long long pre = wave_incl_scan_i64(in ? (long long)rint(scaled(a, E)) : 0ll);
                if (in) mine = sg + (double)pre * u;
                sg = sg + r.val[g];
            }
            st += len;
        }
        if (lane < cnt) P.c[i] = mine;
    }
    __syncthreads();
    FS2_CHAIN_STAMP(4);
}

hipError_t launch_chain(const ChainParams &p, hipStream_t s, hipEvent_t e0) {
    if (p.n <= 0) {
        if (p.total) hipLaunchKernelGGL(k_chain_walk, dim3(1), dim3(1024), 0, s, p);
        return hipGetLastError();
    }
    const unsigned ng = (unsigned)((p.n + 1023) / 1024) + (p.cpart ? kFoldBlocks : 0);
    FS2_LAUNCH_EV(k_chain_units, dim3(ng), dim3(1024), s, e0, nullptr, p);
    hipLaunchKernelGGL(k_chain_walk, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_chain_export(const ChainParams &p, hipStream_t s) {
    if (p.n <= 0) {
        hipLaunchKernelGGL(k_chain_walk, dim3(1), dim3(1024), 0, s, p);
        return hipGetLastError();
    }
    const unsigned ng = (unsigned)((p.n + 1023) / 1024);
    hipLaunchKernelGGL(k_chain_units, dim3(ng), dim3(1024), 0, s, p);
    hipLaunchKernelGGL(k_chain_walk, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_chain_walk_from(const ChainParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_chain_walk, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

// One wave: every shard's ops in shard order (serial fp64 adds, read 64 at a time).
__global__ __launch_bounds__(64) void k_chain_fold(const ChainSummary *all, int32_t world, int32_t shard,
                                                    ShardOrder order, double *total, double *entry,
                                                    DevStats *stats) {
    const int lane = threadIdx.x;
    double s = 0.0, at = 0.0;
    bool over = false;
    for (int q = 0; q < world && !over; ++q) {
        const ChainSummary &S = all[order.r[q]];
        if (q == shard) at = s;
        const int n = S.nops;
        if (n > kChainOpsCap) {
            over = true;
            break;
        }
        for (int k0 = 0; k0 < n; k0 += 64) {
            const double v = (k0 + lane < n) ? S.ops[k0 + lane] : 0.0;
            const int nb = min(64, n - k0);
            for (int j = 0; j < nb; ++j) s = s + bcast(v, j);
        }
    }
    if (lane == 0) {
        if (over) {
            stats->reduce_amb += 1;          // the tree estimates stay: counted, never hidden
            stats->error_flags |= 4;         // (fs2.h: EXACT fails the scan, AUTO reports it)
        } else {
            if (total) *total = s;
            if (entry) *entry = at;
        }
    }
}

hipError_t launch_chain_fold(const ChainSummary *all, int32_t world, int32_t shard, const int8_t *rank_of,
                             double *total, double *entry, DevStats *stats, hipStream_t s) {
    ShardOrder o{};
    for (int q = 0; q < world && q < kMaxRanks; ++q) o.r[q] = rank_of[q];
    hipLaunchKernelGGL(k_chain_fold, dim3(1), dim3(64), 0, s, all, world, shard, o, total, entry, stats);
    return hipGetLastError();
}

// ------------------------------------------------------- numpy sum of w^2 --

#ifdef FS2_PHASE_TIMING
hipError_t debug_chain_times(unsigned long long out[8], int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain), sizeof(unsigned long long) * 8);
    if (e == hipSuccess && reset) {
        unsigned long long z[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_chain), z, sizeof z);
    }
    return e;
}
#endif

int64_t np_sumsq_chunks(int64_t n) { return (n + kNpChunk - 1) / kNpChunk; }

// Sharded exact mode: numpy's chunks of np.sum(w'^2) in the GLOBAL order that
// overlap this shard [first, first + n), one workgroup each.  A chunk held whole
// is summed here (its leaves by 8 lanes each, then its tree); the chunk cut by the
// shard's first (last) boundary is described in rx->head (rx->tail): the sums of
// the leaves held whole, the raw weights of the leaf the boundary cuts
// (k_global_finalize_x completes it with the neighbour's half).  Shards hold at
// least one chunk's worth of particles, so a chunk is cut at most once.
__global__ __launch_bounds__(1024) void k_np_shard(const double *w, int64_t n, int64_t first, int64_t N,
                                                   const NpTailPlan *gtail, RankRecordX *rx) {
    __shared__ double s_w[kNpChunk];
    __shared__ double s_leaf[kNpMaxLeaves];
    const int t = threadIdx.x;
    const int64_t c0 = first / kNpChunk, c1 = (first + n - 1) / kNpChunk;
    const int64_t c = c0 + blockIdx.x;
    const int64_t cs = c * kNpChunk;
    const int m = (int)min<int64_t>(kNpChunk, N - cs);
    const int lo = (int)(max(first, cs) - cs), hi = (int)(min(first + n, cs + m) - cs);
    for (int e = t; e < kNpChunk; e += 1024) s_w[e] = (e >= lo && e < hi) ? w[cs + e - first] : 0.0;
    __syncthreads();
    const int nl = np_chunk_leaves(m, gtail);
    // every leaf held whole: 8 lanes per leaf (numpy's 8 accumulators), one leaf
    // per 8 lanes and round
    for (int L0 = 0; L0 < nl; L0 += 128) {
        const int L = L0 + (t >> 3), k = t & 7;
        const bool in = L < nl;
        const int off = in ? np_leaf_off(m, gtail, L) : 0, len = in ? np_leaf_len(m, gtail, L) : 0;
        const bool whole = in && off >= lo && off + len <= hi;
        double r = 0.0;
        const int full = len - len % 8;
        if (whole && len >= 8) {
            r = s_w[off + k] * s_w[off + k];
            for (int i = 8 + k; i < full; i += 8) r += s_w[off + i] * s_w[off + i];
        }
        r += __shfl_xor(r, 1, 64);
        r += __shfl_xor(r, 2, 64);
        r += __shfl_xor(r, 4, 64);
        if (whole && k == 0) {
            double res = (len < 8) ? 0.0 : r;
            for (int i = (len < 8) ? 0 : full; i < len; ++i) res += s_w[off + i] * s_w[off + i];
            s_leaf[L] = res;
        }
    }
    __syncthreads();
    const int64_t cw0 = (first % kNpChunk == 0) ? c0 : c0 + 1;   // first chunk held whole
    if (lo == 0 && hi == m) {
        if (t == 0) rx->sums[c - cw0] = np_chunk_combine(s_leaf, m, gtail);
    }
    if (t == 0 && blockIdx.x == 0) {
        const int64_t cl = ((first + n) % kNpChunk == 0 || first + n == N) ? c1 : c1 - 1;   // last held whole
        rx->first_chunk = (int32_t)cw0;
        rx->nsums = (int32_t)max<int64_t>(0, cl - cw0 + 1);
    }
    // the edges (thread 0: at most 128 leaves and 127 raw weights each)
    if (t == 0) {
        const bool head = c == c0 && lo > 0, tail = c == c1 && hi < m;
        if (blockIdx.x == 0 && !head) rx->head.chunk = -1;
        if (c == c1 && !tail) rx->tail.chunk = -1;
        for (int side = 0; side < 2; ++side) {
            if (!(side == 0 ? head : tail)) continue;
            NpEdge &E = side == 0 ? rx->head : rx->tail;
            const int p = side == 0 ? lo : hi;      // the cut, chunk-relative
            int kc = 0;
            while (kc + 1 < nl && np_leaf_off(m, gtail, kc + 1) <= p) ++kc;
            const int off = np_leaf_off(m, gtail, kc), len = np_leaf_len(m, gtail, kc);
            const bool inside = p > off && p < off + len;
            E.chunk = (int32_t)c;
            E.cut = inside ? kc : -1;
            if (side == 0) {                         // leaves from the cut on
                const int l0 = (p >= off + len) ? kc + 1 : (inside ? kc + 1 : kc);
                E.leaf0 = l0;
                E.nleaf = nl - l0;
                E.rfrom = inside ? p - off : 0;
                E.nraw = inside ? off + len - p : 0;
            } else {                                 // leaves before the cut
                const int l1 = inside ? kc : ((p >= off + len) ? kc + 1 : kc);
                E.leaf0 = 0;
                E.nleaf = l1;
                E.rfrom = 0;
                E.nraw = inside ? p - off : 0;
            }
            for (int j = 0; j < E.nleaf; ++j) E.leaf[j] = s_leaf[E.leaf0 + j];
            for (int j = 0; j < E.nraw; ++j) E.raw[j] = s_w[off + E.rfrom + j];
        }
    }
}

hipError_t launch_np_shard(const double *w, int64_t n, int64_t first, int64_t n_global, const NpTailPlan *gtail,
                           RankRecordX *rx, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t c0 = first / kNpChunk, c1 = (first + n - 1) / kNpChunk;
    hipLaunchKernelGGL(k_np_shard, dim3((unsigned)(c1 - c0 + 1)), dim3(1024), 0, s, w, n, first, n_global, gtail, rx);
    return hipGetLastError();
}

// numpy's pairwise_sum recursion (loops_utils.h.src) over the partial last chunk
// of n elements: n > 128 splits at n2 = n / 2 rounded down to a multiple of 8;
// leaves in order, internal nodes in post-order.  False when there is none.
bool np_tail_plan(int64_t n, NpTailPlan *out) {
    const int m = (int)(n % kNpChunk);
    *out = NpTailPlan{};
    if (m == 0) return false;
    struct Rec {
        NpTailPlan *p;
        int nodes = 0;
        int go(int off, int len) {            // returns the node index of [off, off + len)
            if (len <= 128) {
                p->off[p->nl] = off;
                p->len[p->nl] = len;
                return p->nl++;
            }
            int n2 = len / 2;
            n2 -= n2 % 8;
            const int l = go(off, n2), r = go(off + n2, len - n2);
            p->a[nodes] = l;
            p->b[nodes] = r;
            return -(++nodes);                // internal: resolved below
        }
    } rec{out};
    // two passes: the first counts the leaves (internal node ids are nl + k)
    rec.go(0, m);
    const int nl = out->nl;
    for (int k = 0; k < rec.nodes; ++k) {
        if (out->a[k] < 0) out->a[k] = nl - out->a[k] - 1;
        if (out->b[k] < 0) out->b[k] = nl - out->b[k] - 1;
    }
    return true;
}

#ifdef FS2_PHASE_TIMING
FS2_TAIL_READER(debug_tail_times_exact)
#endif

}  // namespace fs2
