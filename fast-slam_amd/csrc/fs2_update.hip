// fs2_update.hip -- CDNA4 (gfx950) kernels of the FastSLAM 2.0 particle update
// (reference fast_slam_2/algorithms/fast_slam_2.py:33-223).
//
// Layout in HBM (see fs2_kernels.hpp and DESIGN.md):
//   particle scalars x/y/yaw/w (fp64) and cnt (int32) in logical particle order;
//   landmark maps in 128-byte pages of 8 fp32 gate mirrors, each naming the
//   slot's 48-byte fp64 record in a record pool; particle i's map is row i of
//   the page table pt[row][i]; pages and records are shared after resampling,
//   a page is copied on its first write and a written slot gets a new record
//   (fs2_kernels.hpp).
//
// Kernels
//   k_candidates    streaming fp32 gate-mirror pass listing each particle's
//                   candidate slots for up to kMaxM measurements;
//   k_update        move + exact association + EKF/append + likelihood over the
//                   candidates;
//   k_wsum          weight total (fast_slam_2.py:166);
//   k_normalize     normalise + per-block sum w'^2 / argmax / max count (:161-175);
//   k_finalize      N_eff, resample decision, estimate, u0 (:60-67, :201-223);
//   k_scan_*, k_resample_src, k_plan_*, k_copy_maps, k_gather_particles,
//   k_estimate      low-variance resample (:177-199);
//   k_import/k_export, k_fill, k_iota.
#include "fs2_chain.hpp"

namespace fs2 {

// Optional per-phase wave timing of k_update (build with -DFS2_PHASE_TIMING;
// read back with fs2_debug_phase_times).  Compiled out otherwise.
#ifdef FS2_PHASE_TIMING
__device__ unsigned long long g_phase[8];
#define FS2_PHASE(k)                                                                         \
    do {                                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                           \
        if ((threadIdx.x & 63) == 0 && (k) > 0) atomicAdd(&g_phase[(k) - 1], t_ - ph_last);   \
        ph_last = t_;                                                                        \
    } while (0)
#else
#define FS2_PHASE(k) do { } while (0)
#endif

// ------------------------------------------------------- k_candidates ------
//
// Streaming half of the association (fast_slam_2.py:95-106 first-match search).
// One lane per particle walks its whole map reading only the 16-byte fp32 gate
// mirrors (one 128-byte page = one cache line per lane and group of 8 slots,
// the next group in flight while this one is tested) and lists, in slot order,
// every slot the mirror cannot rule out for at least one measurement of the
// pass, with the slot's record id (so k_update reads the record directly).  No
// fp64, no calls: the kernel stays small enough for full occupancy, which is
// what an HBM stream needs.
//
// Exactness: measurement k can only match slot j in the state slot j had when
// the first measurement matching it arrived, and that first match sees slot j
// unmodified (only matches modify slots), so every slot that will ever match
// passes the conservative mirror test on the pre-scan map.  Slots not listed
// can therefore never match and are never modified; k_update visits exactly the
// listed ones.  A list longer than kMaxCand stores its first kMaxCand entries
// and k_update resumes with an exact scan after the last stored one.
// Measured slower and removed (profiles/r01_v13_ab_k_candidates.txt, history):
// deeper descriptor prefetch, the Euclidean box test on pages that pass the
// bands, the band pre-test on slots of open pages, predicated page loads.
constexpr int kDescAhead = 2;      // page descriptors a lane keeps in flight
constexpr int kCopyBatch = 8;      // copy-on-write pages per lane and batch (8 lanes per page)

static_assert(kMaxCand == 8, "sort8 sorts the candidate list");

// Candidate list entry: slot index (the reference's list position) in the high
// bits, so that entries sort in slot order; page position; record id.
__device__ __forceinline__ uint64_t cand_entry(int slot, int pos, uint32_t rec) {
    return ((uint64_t)slot << 44) | ((uint64_t)pos << 32) | (uint64_t)rec;
}
__device__ __forceinline__ int cand_slot(uint64_t e) { return (int)(e >> 44); }
__device__ __forceinline__ int cand_pos(uint64_t e) { return (int)((e >> 32) & 0xfffu); }
__device__ __forceinline__ uint32_t cand_rec(uint64_t e) { return (uint32_t)e; }

__device__ __forceinline__ void cmpx(uint64_t &a, uint64_t &b) {
    const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}
// Batcher's odd-even merge sort of 8 keys (19 compare-exchanges, branch-free)
__device__ __forceinline__ void sort8(uint64_t (&e)[8]) {
    cmpx(e[0], e[1]); cmpx(e[2], e[3]); cmpx(e[4], e[5]); cmpx(e[6], e[7]);
    cmpx(e[0], e[2]); cmpx(e[1], e[3]); cmpx(e[4], e[6]); cmpx(e[5], e[7]);
    cmpx(e[1], e[2]); cmpx(e[5], e[6]);
    cmpx(e[0], e[4]); cmpx(e[1], e[5]); cmpx(e[2], e[6]); cmpx(e[3], e[7]);
    cmpx(e[2], e[4]); cmpx(e[3], e[5]);
    cmpx(e[1], e[2]); cmpx(e[3], e[4]); cmpx(e[5], e[6]);
}

// __move_particle (fast_slam_2.py:69-87) of local particle i: noisy odometry from
// the injected / numpy draw or Philox(seed, scan, global index), yaw wrapped by
// Python's floor-mod, then the translation along the new yaw.
__device__ __forceinline__ void move_particle(const UpdateParams &P, int64_t i, double &px, double &py,
                                              double &pyaw) {
    const double nz = P.noise ? P.noise[i] : P.sigma * philox_normal(P.seed, P.scan, (uint64_t)(P.gidx0 + i));
    double ntr, nrot;
    if (P.rotation != 0.0) {
        ntr = 0.0;
        nrot = P.rotation + nz;
    } else {
        ntr = P.translation + nz;
        nrot = 0.0;
    }
    pyaw = pymod(pyaw + nrot + kPi, kTwoPi) - kPi;
    px += ntr * cos(pyaw);
    py += ntr * sin(pyaw);
}

template <int MAXM>
__global__ __launch_bounds__(kBlock) void k_candidates(const UpdateParams P) {
    if (P.stats->error_flags & 8) return;     // page_refs: localisation failed, the scan fails
    __shared__ uint64_t s_list[kMaxCand][kBlock];
    __shared__ Band s_band[MAXM];
    __shared__ uint16_t s_rows[kBBoxRows];      // rows the row boxes leave open, ascending
    __shared__ uint8_t s_rmask[kBBoxRows];      // their measurements (the row box's open mask)
    __shared__ int s_wc[kBlock / 64];
    const int tid = threadIdx.x;
    const int64_t n = P.n;
    const int64_t blk = P.blk0 + blockIdx.x;   // this launch may cover a chunk of the blocks
    const int64_t i = blk * kBlock + tid;
    const bool live = i < n;
    MapRef map = P.map;
    const int32_t *cntp = P.cnt;
    double *xp = P.x, *yp = P.y, *yawp = P.yaw;
    if (P.gen) {                               // the current set, read on the device
        const BufSet &b = P.sets[__builtin_amdgcn_readfirstlane(*(volatile const uint32_t *)P.gen) & 1u];
        map.pt = b.pt;
        map.bbox = b.bbox;
        cntp = b.cnt;
        xp = b.x;
        yp = b.y;
        yawp = b.yaw;
    }
    const int c = live ? cntp[i] : 0;
    // The motion sample runs here when its noise is final before this pass
    // (move_cand): association does not read the pose (Q2, the robot-frame point
    // against world landmarks), so the fp64 sample's arithmetic overlaps this
    // kernel's page-line latency instead of k_update's memory stream, which then
    // reads the moved pose.
    if (P.move_cand && live) {
        double px = xp[i], py = yp[i], pyaw = yawp[i];
        move_particle(P, i, px, py, pyaw);
        xp[i] = px;
        yp[i] = py;
        yawp[i] = pyaw;
    }
    const Desc *ptrow = map.pt + (live ? i : 0);
    const float slb = *map.slb;
    if (blockIdx.x == 0 && tid == 0 && P.slb_pass) *P.slb_pass = slb;
    const int rlast = map.rows - 1;
    // Each measurement's band (gate_band): a page whose box, or a slot whose
    // mirror, lies beyond it in x or in y is rejected by integer / one-compare
    // tests; computed once per workgroup, kept in scalar registers.
    if (tid < MAXM) {
        Band b = band_none();
#pragma unroll
        for (int k = 0; k < MAXM; ++k)
            if (tid == k && k < P.m)
                b = gate_band(P.meas.fx[k], P.meas.fy[k], P.meas.fe[k], slb, P.gate2f, map.frame);
        s_band[tid] = b;
    }
    __syncthreads();
    uint32_t bc[MAXM];               // (x a, x b, y a, y b) code thresholds, one byte each
#pragma unroll
    for (int k = 0; k < MAXM; ++k) {
        bc[k] = __builtin_amdgcn_readfirstlane(s_band[k].cx | (s_band[k].cy << 16));
    }
    // the list lives in LDS until the walk ends: (record id << 16 | slot) per
    // entry (a global store inside the walk would serialise the prefetch, since
    // vmcnt counts loads and stores in issue order)
    int nc = 0;
    unsigned visited = 0, groups = 0, opened = 0;

    // Every streamed row's page is opened for the measurements its workgroup row
    // box leaves open (the row test below; without row boxes, all of them): its 8
    // mirrors are loaded by the wave together (lanes past their map read page 0,
    // which stays in cache, and discard it).  (Round 6: per-page boxes in 8-byte
    // descriptors rejected ~1 % of these pages; they are gone.)
    const unsigned all_m = (1u << P.m) - 1u;
    // slots of open page g (mirrors mir) tested against the measurements of om only
    auto test_page = [&](const float4 *mir, int g, unsigned om) {
        const int j0 = g * kPageSlots;
#pragma unroll
        for (int u = 0; u < kScanGroup; ++u) {
            if (j0 + u < c) {
                ++visited;
                const float4 mv = mir[u];
                const float cx = fabsf(mv.x) * 2.3841858e-7f;   // 2^-22 |x_lm|
                const float cy = fabsf(mv.y) * 2.3841858e-7f;
                bool hit = false;
#pragma unroll
                for (int k = 0; k < MAXM; ++k) {
                    if ((om >> k) & 1u) {
                        hit |= !gate_reject_fast(mv, cx, cy, P.meas.fx[k], P.meas.fy[k], P.meas.fe[k],
                                                 P.gate2f);
                    }
                }
                if (hit) {
                    // the kMaxCand smallest slots (an overflowing list still settles every
                    // measurement that matches among them; k_update scans on past them)
                    const uint64_t e = cand_entry(mirror_slot(mv), j0 + u, mirror_rec(mv));
                    if (nc < kMaxCand) {
                        s_list[nc][tid] = e;
                    } else {
                        // (rare: a rolled loop keeps k_candidates' registers at 8 waves)
                        int mq = 0;
                        uint64_t me = s_list[0][tid];
#pragma unroll 1
                        for (int q = 1; q < kMaxCand; ++q) {
                            const uint64_t x = s_list[q][tid];
                            if (x > me) {
                                me = x;
                                mq = q;
                            }
                        }
                        if (e < me) s_list[mq][tid] = e;
                    }
                    ++nc;
                }
            }
        }
    };
    // The rows to stream: those whose workgroup row box some band leaves open
    // (every lane's page box of the row lies inside it, and the band test is
    // monotone in the box, so a rejected row would reject each lane's page);
    // without row boxes, every row.  One thread per row, compacted in row order.
    const bool use_bb = map.bbox != nullptr;
    int nrows = map.rows;
    if (use_bb) {
        unsigned rm = 0u;
        if (tid < map.rows) rm = box_open_mask<MAXM>(map.bbox[blk * kBBoxRows + tid], bc, P.m);
        const bool pass = rm != 0u;
        const uint64_t bm = __ballot(pass);
        const int wid = tid >> 6, lane = tid & 63;
        if (lane == 0) s_wc[wid] = __popcll(bm);
        __syncthreads();
        int off = 0;
        nrows = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) {
            off += (w < wid) ? s_wc[w] : 0;
            nrows += s_wc[w];
        }
        if (pass) {
            const int at = off + __popcll(bm & ((1ull << lane) - 1ull));
            s_rows[at] = (uint16_t)tid;
            s_rmask[at] = (uint8_t)rm;
        }
        __syncthreads();
    }
    // row of list entry q (past the end: row 0, a valid address whose load is discarded)
    auto row_at = [&](int q) -> int { return use_bb ? (q < nrows ? (int)s_rows[q] : 0) : min(q, rlast); };
    Desc dq[kDescAhead];             // descriptors of list entries q .. q + kDescAhead - 1 in flight
#pragma unroll
    for (int q = 0; q < kDescAhead; ++q) dq[q] = ptrow[(int64_t)row_at(q) * n];
    for (int q = 0; q < nrows; ++q) {
        const int g = row_at(q);
        if (!__any(g * kPageSlots < c)) break;      // rows ascend: no lane has more
        const Desc d = dq[0];
#pragma unroll
        for (int u = 0; u + 1 < kDescAhead; ++u) dq[u] = dq[u + 1];
        dq[kDescAhead - 1] = ptrow[(int64_t)row_at(q + kDescAhead) * n];
        if (g * kPageSlots < c) ++groups;
        const unsigned om = (g * kPageSlots < c) ? (use_bb ? (unsigned)s_rmask[q] : all_m) : 0u;
        if (!__any(om)) continue;
        const char *pg = page_ptr(map.pool, om ? d : 0u);
        float4 mir[kScanGroup];
#pragma unroll
        for (int u = 0; u < kScanGroup; ++u) mir[u] = load_mirror(pg, u);
        if (om) {
            ++opened;
            test_page(mir, g, om);
        }
    }
    if (live) {
        P.ncand[i] = nc;
        // pages may hold their slots in any order: the list goes out in slot
        // (reference list) order -- an overflowing list as its kMaxCand smallest
        // slots, after which k_update runs the reference's loop for what is left
        uint64_t e[kMaxCand];
#pragma unroll
        for (int q = 0; q < kMaxCand; ++q) e[q] = (q < nc) ? s_list[q][tid] : ~0ull;
        sort8(e);
#pragma unroll
        for (int q = 0; q < kMaxCand; ++q)
            if (q < nc) P.cand[(int64_t)q * n + i] = e[q];
    }
    // kCWords, kCGroups, kCVisited, kCOpened
    const unsigned cv[4] = {(unsigned)min(nc, kMaxCand), groups, visited, opened};
    // the first pass of a scan stores its counters, later passes add
    block_counters<kBlock, kCWords, 4>(cv, P.cpart, P.nblk, blk, P.k0 == 0 ? 0xffffffffu : 0u, 0.0, nullptr);
}

template <int K>
static __device__ __forceinline__ uint32_t sel_u32(int t, const uint32_t (&a)[K]) {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < K; ++q)
        if (t == q) v = a[q];
    return v;
}

// ------------------------------------------------------------ k_update ------
//
// One lane per particle: move, then the exact association + EKF over the
// candidate slots in slot order.  The M measurements of a scan are sequential
// in the reference (measurement k sees the map left by k-1), but measurement k
// only ever changes the slot it matched or appends at the end.  Walking the
// slots once and, at every slot j, testing the still-unmatched measurements in
// order k = 0..M-1 (an EKF update changes the slot in registers before the
// next measurement tests it) reproduces the sequential result exactly while
// reading each slot once instead of M times.  Slots appended in this scan are
// resolved afterwards in measurement order.  Likelihoods multiply into the
// weight in measurement order, as the reference does.  Without the gate filter
// (or past an overflowing candidate list) every slot takes the exact path.
template <int MAXM>
__global__ __launch_bounds__(kBlock) void k_update(const UpdateParams P) {
    if (P.stats->error_flags & 8) return;     // page_refs: localisation failed, the scan fails
    __shared__ Meas s_ms[MAXM];                 // this pass's measurements
    __shared__ double s_lik[MAXM][kBlock];      // per (measurement, lane) likelihood
    __shared__ int16_t s_idx[MAXM][kBlock];     // per (measurement, lane) association (slot < 4096, -1, -2)
    // per wave: the overflow path's per-measurement answers (phase A), then the
    // page copies' task list (B1) -- the same wave uses them one after the other
    union WaveScratch {
        uint2 cow[64 * (MAXM + 1)];             // (shared page, copy)
        struct {
            int best[MAXM][64], bpos[MAXM][64];
        } ov;
    };
    __shared__ WaveScratch s_ws[kBlock / 64];
    __shared__ float4 s_mv[MAXM][kBlock];       // new mirrors of the slots phase A modified
    __shared__ BoxLds s_bb;                     // this workgroup's row boxes (grown by the writes)

#ifdef FS2_PHASE_TIMING
    unsigned long long ph_last = 0;
#endif
    const int tid = threadIdx.x;
    const int64_t blk = P.blk0 + blockIdx.x;
    const int64_t i = blk * kBlock + tid;
    const bool live = i < P.n;
    const int64_t n = P.n;
    if (tid < MAXM) s_ms[tid] = Meas{P.meas.d[tid], P.meas.b[tid], P.meas.ox[tid], P.meas.oy[tid]};
#pragma unroll
    for (int k = 0; k < MAXM; ++k) s_idx[k][tid] = (int16_t)-2;
    MapRef map = P.map;
    double *xp = P.x, *yp = P.y, *yawp = P.yaw, *wp = P.w;
    int32_t *cntp = P.cnt;
    if (P.gen) {                               // the current set, read on the device
        const BufSet &b = P.sets[__builtin_amdgcn_readfirstlane(*(volatile const uint32_t *)P.gen) & 1u];
        xp = b.x;
        yp = b.y;
        yawp = b.yaw;
        wp = b.w;
        cntp = b.cnt;
        map.pt = b.pt;
        map.bbox = b.bbox;
    }
    if (map.bbox && tid < map.rows) lds_box_set(s_bb, tid, map.bbox[blk * kBBoxRows + tid]);
    __syncthreads();

    double px = 0.0, py = 0.0, pyaw = 0.0, w = 0.0;
    int c = 0;
    if (live) {
        px = xp[i];
        py = yp[i];
        pyaw = yawp[i];
        w = wp[i];
        c = cntp[i];
    }
    const int64_t il = live ? i : 0;
    int nalloc = 0;                  // pages taken from this pass's reservation
    int nrec = 0;                    // records taken from this pass's reservation
    unsigned cow = 0, fresh = 0;
    float smin_w = INFINITY;         // smallest positive s of the mirrors this lane writes (slb)
    uint64_t mods = 0;               // existing slots modified in phase A (16 bits each)
    int nmod = 0;
    // this pass's reserved records (m per lane): phase A stores modified slots into them
    uint32_t frec[MAXM];
#pragma unroll
    for (int t = 0; t < MAXM; ++t) {
        frec[t] = (live && t < P.m) ? P.alloc.rfreel[P.alloc.rbase + (int64_t)t * n + i] : 0u;
    }
    FS2_PHASE(0);
    // __move_particle (fast_slam_2.py:69-87), unless k_candidates moved it
#ifdef FS2_AB_NO_MOVE
    if (false) {                     // A/B timing only (wrong results): the motion sample's share of k_update
#else
    if (live && P.do_move && !P.move_cand) {
#endif
        move_particle(P, i, px, py, pyaw);
    }

    const M2 R{P.R[0], P.R[1], P.R[2], P.R[3]};
    // every descriptor box this lane stores grows the workgroup's row box (an LDS
    // read; atomics only when the row box grows)
    auto box_note = [&](int row, uint32_t b) {
        if (map.bbox) lds_box_merge(s_bb, row, b);
    };
    unsigned pend = live ? ((1u << P.m) - 1u) : 0u;
    unsigned visited = 0, candidates = 0, written = 0, amb = 0, appends = 0;
    bool singular = false;
    const double gate2 = P.gate2;

    FS2_PHASE(1);
    // ---- exact pass over the candidate slots (association + EKF) ----
    int ncl = 0;
    bool overflow = false;
    if (live && P.filter) {
        const int nc = P.ncand[i];
        ncl = min(nc, kMaxCand);
        overflow = nc > kMaxCand;
    }

    // slot `slot` at page position pos (state s): test the pending measurements
    // in order, EKF on a match
    auto visit = [&](int slot, int pos, Slot s) {
        ++candidates;
        bool mod = false;
        M2 I;
        bool ok = inv2(s.P, I);
        singular |= !ok;
        unsigned todo = ok ? pend : 0u;   // measurements still to test at this slot
        while (todo) {
            // test the pending measurements in order; stop at the first match
            int km = -1;
#pragma unroll
            for (int k = 0; k < MAXM; ++k) {
                if (km < 0 && ((todo >> k) & 1u)) {
                    const double qd = quad(I, s_ms[k].ox - s.mx, s_ms[k].oy - s.my);
                    amb += ambiguous(qd, gate2);
                    todo &= ~(1u << k);
                    if (qd >= 0.0 && qd < gate2) km = k;
                }
            }
            if (km < 0) break;
            // one EKF site: the matched measurement sees the slot as left by
            // the earlier measurements (fast_slam_2.py:116-153)
            s_lik[km][tid] = ekf_update(s, px, py, pyaw, s_ms[km], R, singular);
            s_idx[km][tid] = (int16_t)slot;
            pend &= ~(1u << km);
            mod = true;
            ok = inv2(s.P, I);
            singular |= !ok;
            if (!ok) todo = 0u;
        }
        if (mod) {
            // final: every measurement matching the slot was applied above.  Its new
            // record is private, so it is stored now; the mirror naming it goes
            // into the page in phase B (after the page is owned).
            const uint32_t r = sel_u32(nmod, frec);
            store_rec(map.recs, r, s);
            float4 m = with_slot(mirror_of(s), slot);
            m.w = __uint_as_float(r);
            smin_w = fminf(smin_w, mirror_s(m) > 0.0f ? mirror_s(m) : INFINITY);
            s_mv[nmod][tid] = m;
            mods |= (uint64_t)pos << (16 * nmod);
            ++nmod;
            ++written;
        }
    };

    // An overflowing list holds the kMaxCand smallest candidate slots: it settles
    // the measurements that match among them, the overflow scan below only looks
    // past its last slot (`lo`) for the rest.
    int lo = -1;
    int nmod_list = 0;
    {
        // Listed candidates in slot order; the list names their records, so while
        // one is tested the next one's record and the entry after it are in flight
        // (every load is branch-free: a missing entry reads entry 0 and record 0,
        // which are never used).
        const int nl = (pend != 0u) ? ncl : 0;
        auto entry = [&](int p) -> uint64_t { return P.cand[(int64_t)(p < nl ? p : 0) * n + il]; };
        auto rec_of = [&](int p, uint64_t e) -> uint32_t { return p < nl ? cand_rec(e) : 0u; };
        uint64_t e0 = entry(0), e1 = entry(1);
        Slot s0 = load_rec(map.recs, rec_of(0, e0));
        for (int p = 0; p < nl && pend != 0u; ++p) {
            const uint64_t e2 = entry(p + 2);
            const Slot s1 = load_rec(map.recs, rec_of(p + 1, e1));
            visit(cand_slot(e0), cand_pos(e0), s0);
            e0 = e1;
            s0 = s1;
            e1 = e2;
        }
        // Without the filter: every slot, in order (such maps are imported in
        // slot order: position j holds slot j).
        if (!P.filter) {
            for (int j = 0; j < c && pend != 0u; ++j) {
                const float4 mv = load_mirror(page_of(map, j, il), j);
                ++visited;
                visit(mirror_slot(mv), j, load_rec(map.recs, mirror_rec(mv)));
            }
        }
        if (overflow && ncl > 0) lo = cand_slot(P.cand[(int64_t)(ncl - 1) * n + il]);
        nmod_list = nmod;
    }
    if (overflow && pend != 0u) {
        // An overflowing list: the reference's loop (landmark_utils.py:103-117),
        // each pending measurement in order taking the smallest slot index that
        // passes the exact gate with the states the earlier measurements left.
        // One pass over the map (page boxes and pre-scan fp32 mirrors skip what
        // cannot pass) finds, on the pre-scan states, each measurement's smallest
        // matching slot.  Processed in order, that answer stands unless its slot
        // was modified meanwhile (then that measurement alone is rescanned); the
        // slots modified so far are tested with their new states.  A singular
        // covariance counts only below the match, where the reference would meet it.
        const int rows = (c + kPageSlots - 1) / kPageSlots;
        const float slb = P.slb_pass ? *P.slb_pass : *map.slb;
        // each measurement's smallest matching slot and its position live in LDS
        // (registers are k_update's occupancy limit)
#pragma unroll
        for (int k = 0; k < MAXM; ++k) {
            s_ws[tid >> 6].ov.best[k][tid & 63] = INT_MAX;
            s_ws[tid >> 6].ov.bpos[k][tid & 63] = -1;
        }
        int sing = INT_MAX;
        // pre-scan pass over every page (measurements `want`; `skip_mods`: ignore
        // slots modified in this pass)
        auto scan = [&](unsigned want, bool skip_mods) {
            for (int g = 0; g < rows; ++g) {
                const Desc d = *pt_entry(map, g, il);
                // (the row's workgroup box holds this page's mirrors; without row boxes
                // every page is opened)
                const uint32_t rb = map.bbox ? lds_box_get(s_bb, g) : kSumOpen;
                unsigned open = 0u;
#pragma unroll
                for (int k = 0; k < MAXM; ++k)
                    if (((want >> k) & 1u) &&
                        !page_reject(rb, map.frame, slb, P.meas.fx[k], P.meas.fy[k], P.meas.fe[k], P.gate2f))
                        open |= 1u << k;
                if (!open) continue;
                const char *pg = page_ptr(map.pool, d);
                for (int u = 0; u < kPageSlots && g * kPageSlots + u < c; ++u) {
                    const int pos = g * kPageSlots + u;
                    if (skip_mods) {
                        bool modded = false;
#pragma unroll
                        for (int q = 0; q < MAXM; ++q)
                            modded |= q < nmod && (int)((mods >> (16 * q)) & 0xffffu) == pos;
                        if (modded) continue;
                    }
                    const float4 mv = load_mirror(pg, u);
                    const int slot = mirror_slot(mv);
                    if (slot <= lo) continue;          // settled by the list (slot order)
                    const float cx = fabsf(mv.x) * 2.3841858e-7f, cy = fabsf(mv.y) * 2.3841858e-7f;
                    unsigned test = 0u;
#pragma unroll
                    for (int k = 0; k < MAXM; ++k)
                        if (((open >> k) & 1u) && slot < s_ws[tid >> 6].ov.best[k][tid & 63] &&
                            !gate_reject_fast(mv, cx, cy, P.meas.fx[k], P.meas.fy[k], P.meas.fe[k], P.gate2f))
                            test |= 1u << k;
                    if (!test && !(mirror_s(mv) == 0.0f && slot < sing)) continue;
                    const Slot s = load_rec(map.recs, mirror_rec(mv));
                    ++candidates;
                    M2 I;
                    if (!inv2(s.P, I)) {
                        sing = min(sing, slot);
                        continue;
                    }
#pragma unroll
                    for (int k = 0; k < MAXM; ++k) {
                        if ((test >> k) & 1u) {
                            const double qd = quad(I, s_ms[k].ox - s.mx, s_ms[k].oy - s.my);
                            amb += ambiguous(qd, gate2);
                            if (qd >= 0.0 && qd < gate2) {
                                s_ws[tid >> 6].ov.best[k][tid & 63] = slot;
                                s_ws[tid >> 6].ov.bpos[k][tid & 63] = pos;
                            }
                        }
                    }
                }
            }
        };
        scan(pend, false);
        for (int k = 0; k < MAXM; ++k) {
            if (!((pend >> k) & 1u)) continue;
            int t = -1;                            // the pre-scan answer's slot, if modified since
            const int pb = s_ws[tid >> 6].ov.bpos[k][tid & 63];
#pragma unroll
            for (int q = 0; q < MAXM; ++q)
                if (q < nmod && pb >= 0 && (int)((mods >> (16 * q)) & 0xffffu) == pb) t = q;
            if (t >= 0) {
                // rescan this measurement over the unmodified slots
                s_ws[tid >> 6].ov.best[k][tid & 63] = INT_MAX;
                s_ws[tid >> 6].ov.bpos[k][tid & 63] = -1;
                scan(1u << k, true);
            }
            int bk = s_ws[tid >> 6].ov.best[k][tid & 63], pk = s_ws[tid >> 6].ov.bpos[k][tid & 63];
            // the slots modified so far past the list, with their new states (the
            // list's were tested in slot order with the states of their turn)
            int tk = -1;
            for (int q = nmod_list; q < nmod; ++q) {
                const int pos = (int)((mods >> (16 * q)) & 0xffffu);
                const float4 mq = s_mv[q][tid];
                const int slot = mirror_slot(mq);
                if (slot >= bk) continue;
                const Slot s = load_rec(map.recs, sel_u32(q, frec));
                ++candidates;
                M2 I;
                if (!inv2(s.P, I)) {
                    sing = min(sing, slot);
                    continue;
                }
                const double qd = quad(I, s_ms[k].ox - s.mx, s_ms[k].oy - s.my);
                amb += ambiguous(qd, gate2);
                if (qd >= 0.0 && qd < gate2) {
                    bk = slot;
                    pk = pos;
                    tk = q;
                }
            }
            if (sing < bk) singular = true;
            if (pk < 0) continue;
            int t2 = tk;
            if (t2 < 0) {
#pragma unroll
                for (int q = 0; q < MAXM; ++q)
                    if (q < nmod && (int)((mods >> (16 * q)) & 0xffffu) == pk) t2 = q;
            }
            Slot s = load_rec(map.recs, t2 >= 0 ? sel_u32(t2, frec)
                                                : mirror_rec(load_mirror(page_of(map, pk, il), pk)));
            s_lik[k][tid] = ekf_update(s, px, py, pyaw, s_ms[k], R, singular);
            s_idx[k][tid] = (int16_t)bk;
            pend &= ~(1u << k);
            if (t2 < 0) {
                t2 = nmod++;
                mods |= (uint64_t)pk << (16 * t2);
                ++written;
            }
            const uint32_t r = sel_u32(t2, frec);
            store_rec(map.recs, r, s);
            float4 m = with_slot(mirror_of(s), bk);
            m.w = __uint_as_float(r);
            smin_w = fminf(smin_w, mirror_s(m) > 0.0f ? mirror_s(m) : INFINITY);
#pragma unroll
            for (int q = 0; q < MAXM; ++q)
                if (q == t2) s_mv[q][tid] = m;
        }
    }

    FS2_PHASE(2);
    // ---- phase B: every store of this pass.  Stores come last because vmcnt
    // counts loads and stores in issue order: a store ahead of a load makes the
    // wait for that load wait for the store as well. ----

    // Rows this lane writes before the appends: the modified slots' rows, then the
    // row the first append lands in when it is partly filled (later appends start
    // fresh pages).  Their descriptors and this pass's reserved free pages and
    // records are loaded together, before any store.
    constexpr int NR = MAXM + 1;
    const int nrows = nmod + ((pend != 0u && c % kPageSlots != 0) ? 1 : 0);
    int rrow[NR];
    Desc rdesc[NR];
    int canon[NR];                   // first entry with the same row
    unsigned cowm = 0u;              // entries whose page B1 copied (their descriptor changes)
#pragma unroll
    for (int t = 0; t < NR; ++t) {
        rrow[t] = (t < nmod) ? (int)((mods >> (16 * t)) & 0xffffu) / kPageSlots
                             : (t == nmod && t < nrows ? c / kPageSlots : 0);
        rdesc[t] = *pt_entry(map, rrow[t], il);
    }
    uint32_t fpage[MAXM];
#pragma unroll
    for (int t = 0; t < MAXM; ++t)     // the pass reserved m pages per lane
        fpage[t] = t < P.m ? P.alloc.freel[P.alloc.base + (int64_t)t * n + il] : 0u;

    // (B1) own those pages.  The wave lists its shared pages in LDS and copies
    // them together, 8 lanes per 128-byte page and 64 pages per batch (8
    // independent 16-byte loads per lane), the loads of the next batch issued
    // before the stores of this one.
    {
        const int lane = tid & 63, wid = tid >> 6;
        int T = 0;                    // pages listed by the wave so far
#pragma unroll
        for (int t = 0; t < NR; ++t) {
            bool task = false;
            uint32_t src = 0, dst = 0;
            canon[t] = t;
#pragma unroll
            for (int u = 0; u < t; ++u)
                if (canon[t] == t && u < nrows && rrow[u] == rrow[t]) canon[t] = u;
            if (t < nrows && canon[t] == t && !(rdesc[t] & kOwned)) {
                task = true;
                src = rdesc[t] & kIdMask;
                dst = sel_u32(nalloc, fpage);
                ++nalloc;
                rdesc[t] = dst | kOwned;
                cowm |= 1u << t;
                ++cow;
            }
            const uint64_t bm = __ballot(task);
            if (task) s_ws[wid].cow[T + __popcll(bm & ((1ull << lane) - 1ull))] = make_uint2(src, dst);
            T += __popcll(bm);
        }
        // (the owned pages' descriptors reach memory after: B2 stores the modified
        // rows', the appends the partly filled row's; nothing reads them from memory
        // before)
        // the task list is per wave: a wave-level barrier orders its LDS writes and reads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int off = (lane & 7) * 16;
        constexpr int CB = kCopyBatch;
        v4i va[CB];                   // clang vector type: HIP's int4 struct defeats SROA here
        uint32_t da[CB];
        auto load_batch = [&](int base, v4i *v, uint32_t *d) {
#pragma unroll
            for (int u = 0; u < CB; ++u) {
                const uint2 tk = s_ws[wid].cow[min(base + 8 * u + (lane >> 3), T - 1)];
                d[u] = tk.y;
                v[u] = *reinterpret_cast<const v4i *>(page_ptr(map.pool, tk.x) + off);
            }
        };
        auto store_batch = [&](const v4i *v, const uint32_t *d) {
#pragma unroll
            for (int u = 0; u < CB; ++u) {
                *reinterpret_cast<v4i *>(page_ptr(map.pool, d[u]) + off) = v[u];
            }
        };
        for (int base = 0; base < T; base += 8 * CB) {
            load_batch(base, va, da);
            store_batch(va, da);
        }
        __threadfence_block();        // copies land before the slot stores below
    }

    FS2_PHASE(3);
    // (B2) modified slots: their mirrors (computed in phase A) into the owned
    // pages, each growing its row's workgroup box; the descriptors of the rows
    // whose page was copied.
    {
#pragma unroll
        for (int t = 0; t < MAXM; ++t) {
            if (t < nmod) {
                const int j = (int)((mods >> (16 * t)) & 0xffffu);
                uint32_t id = 0;
#pragma unroll
                for (int u = 0; u < NR; ++u)
                    if (u == canon[t]) id = rdesc[u];
                const float4 m = s_mv[t][tid];
                reinterpret_cast<float4 *>(page_ptr(map.pool, id))[j & (kPageSlots - 1)] = m;
                box_note(rrow[t], point_box(m, map.frame));
            }
        }
        nrec = nmod;
#pragma unroll
        for (int t = 0; t < MAXM; ++t)
            if (t < nmod && canon[t] == t && ((cowm >> t) & 1u)) *pt_entry(map, rrow[t], il) = rdesc[t];
    }

    FS2_PHASE(4);
    // ---- measurements that matched nothing: appended slots, in order.  The
    // descriptor of the row being appended into stays in registers (ad) and is
    // stored when the appends leave the row. ----
    int nap = 0;
    int arow = -1;
    Desc ad = 0u;
    bool ad_new = false;             // ad differs from the row's stored descriptor
    if (pend != 0u && c % kPageSlots != 0) {
        // the partly filled last row: owned by B1 (its descriptor stored below if B1 copied it)
        arow = c / kPageSlots;
#pragma unroll
        for (int u = 0; u < NR; ++u)
            if (u == canon[nmod]) {
                ad = rdesc[u];
                ad_new = (cowm >> u) & 1u;
            }
    }
    auto page_at = [&](int j) -> char * {
        return (j / kPageSlots == arow) ? page_ptr(map.pool, ad) : page_of(map, j, il);
    };
    while (pend) {
        const int k = __builtin_ctz(pend);
        pend &= pend - 1u;
        const Meas mk = s_ms[k];
        int hit = -1;
        for (int a = 0; a < nap; ++a) {
            const Slot s = load_slot(map, page_at(c + a), c + a);
            ++candidates;
            M2 I;
            if (!inv2(s.P, I)) {
                singular = true;
                break;
            }
            const double q = quad(I, mk.ox - s.mx, mk.oy - s.my);
            amb += ambiguous(q, gate2);
            if (q >= 0.0 && q < gate2) {
                hit = a;
                break;
            }
        }
        if (hit >= 0) {
            // a slot appended by this pass: page (owned) and record are this lane's own
            const int jh = c + hit;
            char *pg = page_at(jh);
            const uint32_t r = mirror_rec(load_mirror(pg, jh));
            Slot s = load_rec(map.recs, r);
            s_lik[k][tid] = ekf_update(s, px, py, pyaw, mk, R, singular);
            const float4 mv = store_slot(map, pg, jh, s, r, jh);
            smin_w = fminf(smin_w, mirror_s(mv) > 0.0f ? mirror_s(mv) : INFINITY);
            box_note(jh / kPageSlots, point_box(mv, map.frame));
            s_idx[k][tid] = (int16_t)(c + hit);
        } else {
            // new landmark in the world frame (fast_slam_2.py:108-111)
            const Slot s{px + mk.d * cos(pyaw + mk.b), py + mk.d * sin(pyaw + mk.b),
                         M2{P.init_cov[0], P.init_cov[1], P.init_cov[2], P.init_cov[3]}};
            const int ja = c + nap;
            const uint32_t r = sel_u32(nrec, frec);
            ++nrec;
            if (ja % kPageSlots == 0) {
                if (arow >= 0 && ad_new) *pt_entry(map, arow, il) = ad;     // leaving that row
                const uint32_t id = take_page(P.alloc, map.n, il, nalloc);
                arow = ja / kPageSlots;
                const float4 mv = store_slot(map, page_ptr(map.pool, id), ja, s, r, ja);
                smin_w = fminf(smin_w, mirror_s(mv) > 0.0f ? mirror_s(mv) : INFINITY);
                box_note(arow, point_box(mv, map.frame));
                ad = id | kOwned;
                ad_new = true;
                ++fresh;
            } else {
                const float4 mv = store_slot(map, page_ptr(map.pool, ad), ja, s, r, ja);
                smin_w = fminf(smin_w, mirror_s(mv) > 0.0f ? mirror_s(mv) : INFINITY);
                box_note(arow, point_box(mv, map.frame));
            }
            s_idx[k][tid] = (int16_t)-1;
            ++nap;
            ++appends;
        }
        ++written;
    }
    if (arow >= 0 && ad_new) *pt_entry(map, arow, il) = ad;
    c += nap;

    FS2_PHASE(5);
    // likelihoods in measurement order (fast_slam_2.py:159); the reference's
    // first-match scan reads j + 1 landmarks for a match at j, the whole map
    // (as it stood) for an append
    unsigned hits = 0, refv = 0, napp = 0;
#pragma unroll
    for (int k = 0; k < MAXM; ++k) {
        const int ix = s_idx[k][tid];
        if (ix >= 0) {
            w *= s_lik[k][tid];
            ++hits;
            refv += (unsigned)ix + 1u;
        } else if (ix == -1) {
            refv += (unsigned)(c - nap + napp);
            ++napp;
        }
        if (live && P.assoc && k < P.m) P.assoc[(int64_t)(P.k0 + k) * n + i] = ix;
    }

    if (live) {
        if (P.do_move && !P.move_cand) {
            xp[i] = px;
            yp[i] = py;
            yawp[i] = pyaw;
        }
        wp[i] = w;
        cntp[i] = c;
    }

    FS2_PHASE(6);
    // ---- block statistics (every counter) and the weight partial.  The first
    // pass stores, except the counters k_candidates already stored for it ----
    const unsigned cv[kNumCounters] = {0u, 0u, visited, 0u, candidates, written, amb, appends, hits, cow, fresh,
                                       refv, singular ? 1u : 0u};
    const unsigned assign =
        P.k0 != 0 ? 0u
                  : (P.filter ? ~((1u << kCWords) | (1u << kCGroups) | (1u << kCVisited) | (1u << kCOpened))
                              : 0xffffffffu);
    block_counters<kBlock, 0, kNumCounters>(cv, P.cpart, P.nblk, blk, assign, live ? w : 0.0,
                                            P.last_pass ? P.wpart + blk : nullptr);
    // (block_counters' barrier orders every box_note before these reads)
    if (map.bbox && tid < map.rows) map.bbox[blk * kBBoxRows + tid] = lds_box_get(s_bb, tid);
    lower_slb(map.slb, smin_w);
}

hipError_t launch_candidates(const UpdateParams &p, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const unsigned grid = (unsigned)(p.blk1 - p.blk0);
    if (grid == 0 || !p.filter) return hipSuccess;
    FS2_LAUNCH_EV(k_candidates<kMaxM>, dim3(grid), dim3(kBlock), s, e0, e1, p);
    return hipGetLastError();
}

hipError_t launch_update(const UpdateParams &p, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const unsigned grid = (unsigned)(p.blk1 - p.blk0);
    if (grid == 0) return hipSuccess;
    FS2_LAUNCH_EV(k_update<kMaxM>, dim3(grid), dim3(kBlock), s, e0, e1, p);
    return hipGetLastError();
}

// ------------------------------------------------------------ k_localize ---
//
// page_refs mode (fs2_kernels.hpp PeerMaps): before an update pass, every row
// entry naming another rank's page that the pass could read -- its box inside
// some measurement's band (the pages k_candidates opens and, a fortiori, those
// k_update's overflow scan opens: page_reject never keeps a page the bands
// reject) or the partly filled last row (an append writes there) -- is pointed at
// a copy of that page in this rank's pools.  One copy per distinct remote page
// and pass (round 5; round 4 copied it once per row entry, so siblings sharing a
// remote page each copied it with its records: 1.3 GB per scan at G = 8):
//   phase 0  every wanted entry inserts its tagged page id into the table; the
//            lane that claims a key copies the page -- the 8 mirrors, each live
//            slot's record into a fresh record (its mirror renamed) -- into pages
//            and records from the free lists' tails (one atomic per workgroup);
//   phase 1  every wanted entry looks its key up and names the copy, shared
//            (not owned: the first write copies it, as after a resample).
// Rows the workgroup row boxes reject are skipped like k_candidates skips them.
template <int MAXM, int PHASE>
__global__ __launch_bounds__(kBlock) void k_localize(const LocalizeParams P) {
    __shared__ Band s_band[MAXM];
    __shared__ uint16_t s_rows[kBBoxRows];
    __shared__ int s_wc[kBlock / 64];
    __shared__ unsigned long long s_base;
    const int tid = threadIdx.x;
    const int64_t blk = blockIdx.x;
    const int64_t i = blk * kBlock + tid;
    const bool live = i < P.n;
    const MapRef map = P.map;
    const int c = live ? P.cnt[i] : 0;
    if (tid < MAXM) {
        Band b = band_none();
#pragma unroll
        for (int k = 0; k < MAXM; ++k)
            if (tid == k && k < P.m) b = gate_band(P.meas.fx[k], P.meas.fy[k], P.meas.fe[k], *map.slb, P.gate2f, map.frame);
        s_band[tid] = b;
    }
    __syncthreads();
    uint32_t bc[MAXM];
#pragma unroll
    for (int k = 0; k < MAXM; ++k) bc[k] = __builtin_amdgcn_readfirstlane(s_band[k].cx | (s_band[k].cy << 16));
    const bool use_bb = map.bbox != nullptr;
    int nrows = map.rows;
    if (use_bb) {
        bool pass = false;
        if (tid < map.rows) pass = box_open_mask<MAXM>(map.bbox[blk * kBBoxRows + tid], bc, P.m) != 0u;
        const uint64_t bm = __ballot(pass);
        const int wid = tid >> 6, lane = tid & 63;
        if (lane == 0) s_wc[wid] = __popcll(bm);
        __syncthreads();
        int off = 0;
        nrows = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) {
            off += (w < wid) ? s_wc[w] : 0;
            nrows += s_wc[w];
        }
        if (pass) s_rows[off + __popcll(bm & ((1ull << lane) - 1ull))] = (uint16_t)tid;
        __syncthreads();
    }
    const int arow = (c % kPageSlots) ? c / kPageSlots : -1;     // an append may write this row
    auto row_at = [&](int q) -> int { return use_bb ? (int)s_rows[q] : q; };
    // (the rows streamed below are those the row boxes leave open -- every row
    // without row boxes -- so a remote page in one is one the pass may open)
    auto wanted = [&](int r, const Desc &d) -> bool { return r * kPageSlots < c && ref_tag(d) != 0u; };
    // every wanted entry of this lane: the open rows' remote pages, then the append
    // row when it is remote and not among them
    auto for_wanted = [&](auto &&fn) {
        if (!live) return;
        bool arow_seen = false;
        for (int q = 0; q < nrows; ++q) {
            const int r = row_at(q);
            if (r * kPageSlots >= c) continue;
            const Desc d = *pt_entry(map, r, i);
            if (wanted(r, d)) {
                fn(r, d);
                arow_seen |= r == arow;
            }
        }
        if (arow >= 0 && !arow_seen) {
            const Desc d = *pt_entry(map, arow, i);
            if (ref_tag(d) != 0u) fn(arow, d);
        }
    };
    const unsigned long long ep = (unsigned long long)P.epoch << 32;
    const uint64_t mask = (uint64_t)P.cap - 1u;
    auto slot0 = [&](uint32_t x) -> uint64_t { return ((uint64_t)x * 0x9E3779B97F4A7C15ull >> 20) & mask; };
    if (PHASE == 1) {
        // every wanted entry names its page's copy (claimed and filled by phase 0)
        unsigned long long rows = 0;
        for_wanted([&](int r, const Desc &d) {
            const unsigned long long want = ep | d;
            uint64_t s = slot0(d);
            for (int64_t probe = 0; probe < P.cap; ++probe, s = (s + 1) & mask)
                if (P.key[s] == want) {
                    const uint32_t id = P.val[s];
                    if (!(id & 0x80000000u)) {        // (0xffffffff: the copy failed, left remote)
                        *pt_entry(map, r, i) = id;
                        ++rows;
                    }
                    break;
                }
        });
        unsigned long long tot = rows;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if ((tid & 63) == 0 && tot) atomicAdd(&P.stats->loc_rows, tot);
        return;
    }
    // phase 0: claim the keys (the claimer's particle index, high bit set, in val:
    // a lane claims a key at most once -- its rows name distinct pages), count them
    const uint32_t marker = 0x80000000u | (uint32_t)i;
    auto find = [&](uint32_t x, bool claim) -> int64_t {     // slot of key x (claim: insert it)
        const unsigned long long want = ep | x;
        uint64_t s = slot0(x);
        for (int64_t probe = 0; probe < P.cap;) {
            const unsigned long long cur = __atomic_load_n(&P.key[s], __ATOMIC_RELAXED);
            if (cur == want) return (int64_t)s;
            if (claim && (cur >> 32) != P.epoch) {             // a slot of an older pass: free
                if (atomicCAS(&P.key[s], cur, want) == cur) {
                    P.val[s] = marker;
                    return -2 - (int64_t)s;                    // claimed by this lane
                }
                continue;                                      // taken meanwhile: look again
            }
            s = (s + 1) & mask;
            ++probe;
        }
        return -1;
    };
    int need = 0;
    for_wanted([&](int, const Desc &d) {
        if (find(d, true) <= -2) ++need;
    });
    // this workgroup's pages: one atomic, then each lane's run
    const int wid = tid >> 6, lane = tid & 63;
    int incl = need;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    __syncthreads();
    if (lane == 63) s_wc[wid] = incl;
    __syncthreads();
    int woff = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        woff += (w < wid) ? s_wc[w] : 0;
        tot += s_wc[w];
    }
    if (tid == 0) {
        s_base = tot ? atomicAdd(&P.stats->loc_pages, (unsigned long long)tot) : 0ull;
        if (tot) atomicAdd(&P.stats->loc_recs, (unsigned long long)tot * kPageSlots);
        // the tails would run into this scan's reservations: nothing localised, the
        // pass's update kernels exit, the scan reports it (never a remote page read
        // through the local pool)
        if (tot && ((int64_t)(s_base + tot) > P.pcap || (int64_t)(s_base + tot) * kPageSlots > P.rcap)) {
            atomicOr(&P.stats->error_flags, 8);
            s_base = ~0ull;
        }
    }
    __syncthreads();
    if (!need) return;
    const bool failed = s_base == ~0ull;
    int64_t k = (int64_t)s_base + woff + incl - need;            // this lane's first localised page
    for_wanted([&](int r, const Desc &d) {
        const int64_t slot = find(d, false);
        if (slot < 0 || P.val[slot] != marker) return;          // another lane's copy
        if (failed) {                                            // (phase 1 leaves the entry remote)
            P.val[slot] = 0xffffffffu;
            return;
        }
        const uint32_t tg = ref_tag(d);
        const float4 *src = reinterpret_cast<const float4 *>(map.peers->pool[tg - 1] + (int64_t)ref_id(d) * kPageBytes);
        const char *srecs = map.peers->recs[tg - 1];
        const uint32_t id = P.freel[P.ftail - 1 - k];
        // every row naming a page holds the same slots of it (sharers of a page have
        // the same map length up to its row: an append to a shared page copies it)
        const int valid = min(kPageSlots, c - r * kPageSlots);
        float4 mv[kPageSlots];
#pragma unroll
        for (int u = 0; u < kPageSlots; ++u) mv[u] = src[u];
        Slot sl[kPageSlots];
#pragma unroll
        for (int u = 0; u < kPageSlots; ++u) sl[u] = load_rec(srecs, u < valid ? mirror_rec(mv[u]) : mirror_rec(mv[0]));
        float4 *dst = reinterpret_cast<float4 *>(page_ptr(map.pool, id));
#pragma unroll
        for (int u = 0; u < kPageSlots; ++u) {
            if (u < valid) {
                const uint32_t rid = P.rfreel[P.rtail - 1 - (kPageSlots * k + u)];
                double2 *q = reinterpret_cast<double2 *>(map.recs + (int64_t)rid * kRecBytes);
                q[0] = make_double2(sl[u].mx, sl[u].my);
                q[1] = make_double2(sl[u].P.a00, sl[u].P.a01);
                q[2] = make_double2(sl[u].P.a10, sl[u].P.a11);
                mv[u].w = __uint_as_float(rid);
            } else {
                mv[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);         // past the map: no record named
            }
            dst[u] = mv[u];
        }
        P.val[slot] = id;
        ++k;
    });
}

hipError_t launch_localize(const LocalizeParams &p, hipStream_t s) {
    if (p.nblk <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_localize<kMaxM, 0>), dim3((unsigned)p.nblk), dim3(kBlock), 0, s, p);
    hipLaunchKernelGGL((k_localize<kMaxM, 1>), dim3((unsigned)p.nblk), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------ generator test hooks --

__global__ __launch_bounds__(kBlock) void k_debug_philox(int64_t n, const uint32_t *ctr, const uint32_t *key,
                                                         uint32_t *out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const U4 r = philox(U4{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]}, key[2 * i], key[2 * i + 1]);
    out[4 * i] = r.x;
    out[4 * i + 1] = r.y;
    out[4 * i + 2] = r.z;
    out[4 * i + 3] = r.w;
}

__global__ __launch_bounds__(kBlock) void k_debug_normals(uint64_t seed, uint64_t stream, uint64_t first, int64_t n,
                                                          double *out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = philox_normal(seed, stream, first + (uint64_t)i);
}

hipError_t launch_debug_philox(int64_t n, const uint32_t *ctr, const uint32_t *key, uint32_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_philox, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, ctr, key,
                       out);
    return hipGetLastError();
}

hipError_t launch_debug_normals(uint64_t seed, uint64_t stream, uint64_t first, int64_t n, double *out,
                                hipStream_t s) {
    hipLaunchKernelGGL(k_debug_normals, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, seed, stream,
                       first, n, out);
    return hipGetLastError();
}

// ------------------------------------------------------- normalise & N_eff --

// Weight total (Python builtin sum in particle order in sequential mode) in
// workgroup 0, and the update pass's block counters folded into the scan
// statistics by workgroups 1 .. kFoldBlocks, each over a slice of the
// columns (atomics into DevStats: integer sums, order-free), in parallel.
__global__ __launch_bounds__(1024) void k_wsum(const ReduceParams P) {
    __shared__ double lds[16];
    __shared__ unsigned long long s_c[16][kNumCounters];
    if (blockIdx.x > 0) {
        fold_counters(P.cpart, P.nwpart, P.stats, blockIdx.x - 1, s_c);
        return;
    }
    if (P.sequential) {
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int64_t i = 0; i < P.n; ++i) t += P.w[i];
            P.stats->total = t;
        }
        return;
    }
    double v = 0.0;
    for (int k = threadIdx.x; k < P.nwpart; k += 1024) v += P.wpart[k];
    const double t = block_sum<1024>(v, lds);
    if (threadIdx.x == 0) P.stats->total = t;
}

hipError_t launch_wsum(const ReduceParams &p, hipStream_t s, hipEvent_t e0) {
    FS2_LAUNCH_EV(k_wsum, dim3(1 + kFoldBlocks), dim3(1024), s, e0, nullptr, p);
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_normalize(const ReduceParams P) {
    __shared__ double s_sq[kBlock / 64], s_bv[kBlock / 64], s_w[kBlock / 64];
    __shared__ int64_t s_bi[kBlock / 64];
    __shared__ int s_mc[kBlock / 64];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool live = i < P.n;
    const double total = P.stats->total;
    double w = 0.0;
    int c = 0;
    if (live) {
        w = P.w[i];
        c = P.cnt[i];
        if (total < P.floor) w = 1.0 / (double)P.n_global;
        else w = (w < P.floor) ? w : w / total;
        P.w[i] = w;
    }
    // exact: this block's two numpy leaves (fs2_exact.hip: 128 elements, 8
    // accumulators of 16 squares added in order, combined ((r0 + r1) + (r2 + r3)) +
    // ((r4 + r5) + (r6 + r7))) when they lie in a full 8192-element chunk;
    // k_finalize adds them up the chunk trees
    if (P.np_leaf && ((int64_t)blockIdx.x + 1) * kBlock <= (P.n / kNpChunk) * kNpChunk) {
        __shared__ double s_sq2[kBlock];
        s_sq2[threadIdx.x] = w * w;
        __syncthreads();
        if (threadIdx.x < 16) {
            const int g = threadIdx.x >> 3, k = threadIdx.x & 7;
            double r = s_sq2[g * 128 + k];
#pragma unroll
            for (int q = 1; q < 16; ++q) r += s_sq2[g * 128 + 8 * q + k];
            r += __shfl_xor(r, 1, 64);
            r += __shfl_xor(r, 2, 64);
            r += __shfl_xor(r, 4, 64);
            if (k == 0) P.np_leaf[(int64_t)blockIdx.x * 2 + g] = r;
        }
    }
    // block_sum / block_argmax / block_max_i (same trees) with one barrier
    const double sq = wave_sum(live ? w * w : 0.0);
    const double ws = P.part_w ? wave_sum(w) : 0.0;
    double bv = live ? w : -INFINITY;
    int64_t bi = live ? i : INT64_MAX;
    wave_argmax(bv, bi);
    const int mc = wave_max_i(c);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        s_sq[wid] = sq;
        s_w[wid] = ws;
        s_bv[wid] = bv;
        s_bi[wid] = bi;
        s_mc[wid] = mc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        double v = s_bv[0];
        int64_t ix = s_bi[0];
        int m = s_mc[0];
#pragma unroll
        for (int k = 0; k < kBlock / 64; ++k) t += s_sq[k];
#pragma unroll
        for (int k = 1; k < kBlock / 64; ++k) {
            argmax_combine(v, ix, s_bv[k], s_bi[k]);
            m = max(m, s_mc[k]);
        }
        P.part_sq[blockIdx.x] = t;
        if (P.part_w) P.part_w[blockIdx.x] = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);   // an estimate only
        P.part_best_w[blockIdx.x] = v;
        P.part_best_i[blockIdx.x] = ix;
        P.part_maxcnt[blockIdx.x] = m;
    }
}

// Exact mode: normalise (fast_slam_2.py:161-175) and, in the same pass, the terms
// of np.sum(weights ** 2) (:219) by numpy's own trees.  numpy sums 8192-weight
// chunks pairwise (the chunk sums then in order); an 8192 chunk's tree is the sum
// of its two 4096 halves, each a balanced tree of 32 leaves of 128 (8 accumulators
// of 16 squares added in order, combined ((r0 + r1) + (r2 + r3)) + ((r4 + r5) +
// (r6 + r7))).  So workgroup b < 2 nfull takes half-chunk b (4 weights per thread,
// loaded and stored as 32-byte runs) and leaves its half sum in np_part[b]; a
// partial last chunk (numpy's recursion, np_tail) is one workgroup with 8 weights
// per thread.  Per workgroup also: the first maximum with its pose (part_best_*,
// part_pose: no dependent load left for k_finalize_chunked), the largest map
// (part_maxcnt), and the sum of every 256 weights (part_w: the resample chain's
// block estimates).  One pass over the weights instead of k_normalize + the leaf
// trees of k_finalize.
template <int EPT>
__device__ __forceinline__ void normalize_span(const ReduceParams &P, int64_t e0, bool tree, double *s_sq,
                                               double *s_leaf, double *s_bv, int64_t *s_bi, int *s_mc,
                                               double &chunk_out, double (&pose_out)[3]) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int64_t n = P.n;
    const int64_t b0 = e0 + (int64_t)EPT * t;            // this thread's first weight
    const double total = P.stats->total;
    double w[EPT];
    int cn[EPT];
    if (b0 + EPT <= n) {
        const double2 *wp = reinterpret_cast<const double2 *>(P.w + b0);
        const int4 *cp = reinterpret_cast<const int4 *>(P.cnt + b0);
#pragma unroll
        for (int h = 0; h < EPT / 2; ++h) {
            const double2 v = wp[h];
            w[2 * h] = v.x;
            w[2 * h + 1] = v.y;
        }
#pragma unroll
        for (int h = 0; h < EPT / 4; ++h) {
            const int4 v = cp[h];
            cn[4 * h] = v.x;
            cn[4 * h + 1] = v.y;
            cn[4 * h + 2] = v.z;
            cn[4 * h + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            w[j] = (b0 + j < n) ? P.w[b0 + j] : 0.0;
            cn[j] = (b0 + j < n) ? P.cnt[b0 + j] : 0;
        }
    }
    double ws = 0.0, bv = -INFINITY;
    int64_t bi = INT64_MAX;
    int mc = 0;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const bool live = b0 + j < n;
        double v = w[j];
        if (total < P.floor) v = 1.0 / (double)P.n_global;
        else v = (v < P.floor) ? v : v / total;
        w[j] = live ? v : 0.0;
        ws += w[j];
        if (live && v > bv) {                    // ascending index: the first maximum stays
            bv = v;
            bi = b0 + j;
        }
        mc = max(mc, live ? cn[j] : 0);
        if (tree) s_sq[EPT * t + j] = w[j] * w[j];
    }
    if (b0 + EPT <= n) {
        double2 *wp = reinterpret_cast<double2 *>(P.w + b0);
#pragma unroll
        for (int h = 0; h < EPT / 2; ++h) wp[h] = make_double2(w[2 * h], w[2 * h + 1]);
    } else {
#pragma unroll
        for (int j = 0; j < EPT; ++j)
            if (b0 + j < n) P.w[b0 + j] = w[j];
    }
    // the resample chain's estimate of each 256-weight block (256 / EPT threads)
    {
        double v = ws;
#pragma unroll
        for (int o = 1; o < kBlock / EPT; o <<= 1) v += __shfl_xor(v, o, 64);
        const int64_t blk = b0 / kBlock;
        if ((t & (kBlock / EPT - 1)) == 0 && blk * kBlock < n && P.part_w) P.part_w[blk] = v;
    }
    wave_argmax(bv, bi);
    mc = wave_max_i(mc);
    if (lane == 0) {
        s_bv[wid] = bv;
        s_bi[wid] = bi;
        s_mc[wid] = mc;
    }
    __syncthreads();                             // s_sq, s_bv written (global w' too)
    // the workgroup's first maximum, and its pose requested before the tree below
    double v = s_bv[0];
    int64_t ix = s_bi[0];
    int m = s_mc[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        argmax_combine(v, ix, s_bv[k], s_bi[k]);
        m = max(m, s_mc[k]);
    }
    if (t == 0 && ix != INT64_MAX) {
        pose_out[0] = P.x[ix];
        pose_out[1] = P.y[ix];
        pose_out[2] = P.yaw[ix];
    }
    double chunk = 0.0;
    if (tree) {
        // accumulator k of leaf L: the leaf's squares 8 q + k, q = 0..15, added in order
        constexpr int NL = 1024 * EPT / 128;     // leaves
        if (t < 8 * NL) {
            const int L = t >> 3, k = t & 7;
            const double *q0 = s_sq + 128 * L + k;
            double r = q0[0];
#pragma unroll
            for (int q = 1; q < 16; ++q) r += q0[8 * q];
            r += __shfl_xor(r, 1, 64);
            r += __shfl_xor(r, 2, 64);
            r += __shfl_xor(r, 4, 64);
            if (k == 0) s_leaf[L] = r;
        }
        __syncthreads();
        // the leaves as a balanced tree in order (DPP rows of 16, then row pairs;
        // lanes past the leaves add +0)
        if (wid == 0) chunk = lane63(dpp_scan(lane < NL ? s_leaf[lane] : 0.0, 0.0,
                                              [](double a, double b) { return a + b; }));
    } else if (wid == 0 && P.np_tail) {
        chunk = np_pairwise_wave(P.w + e0, P.np_tail);   // this workgroup's own stores, after the barrier
    }
    if (t == 0) {
        chunk_out = chunk;
        P.part_best_w[blockIdx.x] = v;
        P.part_best_i[blockIdx.x] = ix;
        P.part_maxcnt[blockIdx.x] = m;
    }
}

__global__ __launch_bounds__(1024) void k_normalize_chunks(const ReduceParams P) {
    __shared__ double s_sq[1024 * 4];            // squares of the half chunk, in weight order
    __shared__ double s_leaf[64];
    __shared__ double s_bv[16];
    __shared__ int64_t s_bi[16];
    __shared__ int s_mc[16];
    FS2_TS_DECL;
    FS2_TS(16, 0);
    const int64_t nfull = P.n / kNpChunk;
    double chunk = 0.0, pose[3] = {0.0, 0.0, 0.0};
    if ((int64_t)blockIdx.x < 2 * nfull)
        normalize_span<4>(P, (int64_t)blockIdx.x * (kNpChunk / 2), true, s_sq, s_leaf, s_bv, s_bi, s_mc, chunk, pose);
    else
        normalize_span<8>(P, nfull * kNpChunk, false, s_sq, s_leaf, s_bv, s_bi, s_mc, chunk, pose);
    FS2_TS(16, 1);
    if (threadIdx.x == 0) {
        P.np_part[blockIdx.x] = chunk;
        P.part_pose[3 * (int64_t)blockIdx.x] = pose[0];
        P.part_pose[3 * (int64_t)blockIdx.x + 1] = pose[1];
        P.part_pose[3 * (int64_t)blockIdx.x + 2] = pose[2];
    }
}

int32_t normalize_chunk_parts(int64_t n) {
    return (int32_t)(2 * (n / kNpChunk) + ((n % kNpChunk) ? 1 : 0));
}

hipError_t launch_normalize_chunks(const ReduceParams &p, hipStream_t s) {
    const unsigned grid = (unsigned)normalize_chunk_parts(p.n);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_normalize_chunks, dim3(grid), dim3(1024), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_normalize(const ReduceParams &p, hipStream_t s) {
    const unsigned grid = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_normalize, dim3(grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------ state import/export --

// stage: [count][lm_cap][6] -> maps of particles first .. first+count-1, written
// into fresh pages and records (row k of particle p takes reserved page
// k * count + p, slot j reserved record j * count + p: row-major, so a wave's
// 64 particles read one row's pages and one slot's records from adjacent ids);
// the pages and records they replace are reclaimed by the next collection.
__global__ __launch_bounds__(kBlock) void k_import(const double *stage, const int32_t *cnt_stage,
                                                   int64_t first, int64_t count, int32_t lm_cap,
                                                   MapRef map, PageAlloc alloc, int32_t rows_each,
                                                   int32_t *cnt, uint32_t *ext, const int32_t *perm,
                                                   int32_t perm_len) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t total = count * lm_cap;
    float smin = INFINITY, amax = 0.0f;
    for (int64_t e = t; e < total; e += (int64_t)gridDim.x * kBlock) {
        const int64_t p = e / lm_cap;
        const int j = (int)(e % lm_cap);
        const int c = cnt_stage[p];
        if (j == 0) cnt[first + p] = c;
        if (j >= c) continue;
        // position j holds slot perm[j] (a spatial layout, fs2_set_state), or slot j
        const int slot = (perm && c == perm_len) ? perm[j] : j;
        const int row = j / kPageSlots;
        // row-major over the chunk's particles: the pages (and records) a wave reads
        // for one row (slot) of 64 consecutive particles are adjacent in the pools
        const uint32_t id = alloc.freel[alloc.base + (int64_t)row * count + p];
        if (j % kPageSlots == 0) *pt_entry(map, row, first + p) = id | kOwned;
        const double *s = stage + (p * lm_cap + slot) * 6;
        const float4 mv = store_slot(map, page_ptr(map.pool, id), j, Slot{s[0], s[1], M2{s[2], s[3], s[4], s[5]}},
                                     alloc.rfreel[alloc.rbase + (int64_t)j * count + p], slot);
        smin = fminf(smin, mirror_s(mv) > 0.0f ? mirror_s(mv) : INFINITY);
        if (isfinite(mv.x)) amax = fmaxf(amax, fabsf(mv.x));
        if (isfinite(mv.y)) amax = fmaxf(amax, fabsf(mv.y));
    }
    lower_slb(map.slb, smin);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    if ((threadIdx.x & 63) == 0 && amax > 0.0f) atomicMax(ext, __float_as_uint(amax));
}

__global__ __launch_bounds__(kBlock) void k_export(double *stage, int64_t first, int64_t count,
                                                   int32_t lm_cap, MapRef map, const int32_t *cnt) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t total = count * lm_cap;
    for (int64_t e = t; e < total; e += (int64_t)gridDim.x * kBlock) {
        const int64_t p = e / lm_cap;
        const int j = (int)(e % lm_cap);
        if (j >= cnt[first + p]) continue;
        // position j holds slot mirror_slot (a remote page: its rank's pools)
        const uint32_t pe = *pt_entry(map, j / kPageSlots, first + p);
        const float4 mv = load_mirror(page_ptr_any(map, pe), j);
        const Slot s = load_rec(recs_of(map, pe), mirror_rec(mv));
        double *d = stage + (p * lm_cap + mirror_slot(mv)) * 6;
        d[0] = s.mx; d[1] = s.my;
        d[2] = s.P.a00; d[3] = s.P.a01; d[4] = s.P.a10; d[5] = s.P.a11;
    }
}

static unsigned grid_for(int64_t total) {
    int64_t g = (total + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    return (unsigned)(g > 0 ? g : 1);
}

hipError_t launch_import(const double *stage, const int32_t *cnt_stage, int64_t first,
                         int64_t count, int32_t lm_cap, MapRef map, PageAlloc alloc,
                         int32_t rows_each, int32_t *cnt, uint32_t *ext, const int32_t *perm,
                         int32_t perm_len, hipStream_t s) {
    hipLaunchKernelGGL(k_import, dim3(grid_for(count * lm_cap)), dim3(kBlock), 0, s, stage,
                       cnt_stage, first, count, lm_cap, map, alloc, rows_each, cnt, ext, perm, perm_len);
    return hipGetLastError();
}


hipError_t launch_export(double *stage, int64_t first, int64_t count, int32_t lm_cap, MapRef map,
                         const int32_t *cnt, hipStream_t s) {
    hipLaunchKernelGGL(k_export, dim3(grid_for(count * lm_cap)), dim3(kBlock), 0, s, stage, first,
                       count, lm_cap, map, cnt);
    return hipGetLastError();
}

__global__ void k_fill(double *p, double v, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (int64_t e = t; e < n; e += (int64_t)gridDim.x * kBlock) p[e] = v;
}

hipError_t launch_fill(double *p, double v, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_fill, dim3(grid_for(n)), dim3(kBlock), 0, s, p, v, n);
    return hipGetLastError();
}

__global__ void k_iota(uint32_t *p, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (int64_t e = t; e < n; e += (int64_t)gridDim.x * kBlock) p[e] = (uint32_t)e;
}

hipError_t launch_iota(uint32_t *p, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kBlock), 0, s, p, n);
    return hipGetLastError();
}

__global__ void k_iota_from(uint32_t *p, uint32_t v0, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (int64_t e = t; e < n; e += (int64_t)gridDim.x * kBlock) p[e] = v0 + (uint32_t)e;
}

hipError_t launch_iota_from(uint32_t *p, uint32_t v0, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_iota_from, dim3(grid_for(n)), dim3(kBlock), 0, s, p, v0, n);
    return hipGetLastError();
}

#ifdef FS2_PHASE_TIMING
hipError_t debug_phase_times(unsigned long long out[8], int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * 8);
    if (e == hipSuccess && reset) {
        unsigned long long z[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z);
    }
    return e;
}
#endif

#ifdef FS2_PHASE_TIMING
FS2_TAIL_READER(debug_tail_times_update)
#endif

}  // namespace fs2
