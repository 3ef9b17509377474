// fs2_kernels.hpp -- kernel parameter blocks and launch wrappers shared by
// fs2_kernels.hip (device code) and fs2_api.hip (host C-ABI).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace fs2 {

constexpr int kBlock = 256;          // 4 waves of 64
constexpr int kPageSlots = 8;        // landmark slots per page
constexpr int kMaxSlots = 4096;      // landmark slots per particle max
constexpr int kMaxRows = kMaxSlots / kPageSlots;   // page-table rows max
constexpr int kMaxM = 4;             // measurements fused into one map pass
constexpr int kScanGroup = kPageSlots;   // slots whose mirrors a lane loads per step (128 B)
constexpr int kMaxCand = 8;          // candidate slots listed per particle and pass

// A page holds 8 consecutive slots of a map as their gate mirrors, one 128-byte
// line: 8 x {float x, float y, float s, uint32 rec}.  rec names the slot's fp64
// record (x, y, P00, P01, P10, P11; 48 B) in the record pool.  Records are
// immutable and shared like pages: a slot write stores a new record and points
// the (private) page's mirror at it, so copy-on-write moves 128 B, not the slots.
// Pages live in one pool (page id p at pool + 128 p).  A map is a row of 4-byte
// page descriptors in the page table pt[row][particle] (Desc = uint32): the page
// id; bit 31 says the map owns the page (no other entry refers to it) and may
// write it in place, otherwise the first write copies the page (copy-on-write).
// Resampling shares pages instead of copying maps, and copies 4 bytes per row.
// Boxes (bounding boxes on the handle's summary grid, rounded outward: four 8-bit
// cell codes x lo, x hi, y lo, y hi; SumFrame) live per workgroup row (bbox
// below), not per page (round 6: a per-page box in an 8-byte descriptor rejected
// ~1 % of the rows the row boxes stream, for twice the resample's row copy).
// With the handle-wide lower bound slb on every nonzero mirror s, a box lets the
// candidate stream reject a whole row with one test that is never less
// conservative than the slot tests it replaces (page_reject); an s = 0 slot
// makes its row's box unbounded (never rejected).
constexpr int kPageBytes = 128;
constexpr int kRecBytes = 48;   // 64-byte records measured slower (profiles/r03_ab_rec64.txt)
constexpr uint32_t kOwned = 0x80000000u;
constexpr uint32_t kIdMask = 0x7fffffffu;
constexpr uint32_t kRecIdLimit = 0xffffffffu;   // record ids are uint32 (mirror .w, free lists)
typedef uint32_t Desc;
// A descriptor with a box, as the sharded transfers carry it (.x entry, .y box:
// the page's own box, or its source workgroup's row box)
typedef uint2 XDesc;

// Summary grid: box bound codes c in [0, 255]; lo(c) = org + (c - 1) cell (c = 0:
// unbounded), hi(c) = org + c cell (c = 255: unbounded).  cell is a power of two
// and org a multiple of it, so every bound is exact in fp32.
struct SumFrame {
    float org, cell;
    float icell;             // 1 / cell, rounded (informational: codes are computed against the exact bounds)
};
constexpr uint32_t kSumOpen = 0xff00ff00u;   // unbounded box: never rejected

// Workgroup row boxes: bbox[b * kBBoxRows + r] is a box (same codes) holding
// every live slot mirror of row r's pages of every particle of workgroup b
// (particles [256 b, 256 b + 256)).  k_candidates tests it against the
// measurement bands once per workgroup and streams only the rows it cannot
// reject, so most descriptors are never read.  Boxes only grow between rebuilds
// (k_update merges each mirror it writes; a resample unions its sources'
// workgroups' boxes; imports rebuild them from the pages); maps of more than
// kBBoxRows rows run without (every page of every row is opened).
constexpr int kBBoxRows = 256;
constexpr uint32_t kBoxEmpty = 0x00ff00ffu;  // x lo = y lo = 255, x hi = y hi = 0: holds nothing

// Counters of the update pass, kept per workgroup (cpart[counter][block]: the
// first pass of a scan stores them, later passes add) and folded into DevStats
// by k_wsum: no same-address atomics on the hot kernels.
// k_candidates adds [kCWords, kCOpened], k_update [kCVisited, kCSingular].
enum : int {
    kCWords, kCGroups, kCVisited, kCOpened, kCCandidates, kCWritten, kCAmbiguous, kCAppends, kCHits, kCCow, kCNew,
    kCRefVisits, kCSingular, kNumCounters
};

// Device statistics of one scan (zeroed before every scan).
// A wave of k_ranges whose sources have more than kWaveFill outputs in all lists
// them for k_fill_runs in pieces of kFillChunk instead of filling them 64 per step
// (Q10: when the normalised weights sum below 1 the last particle takes every
// output past their total -- a third of 10^6 outputs in the appended-maps workload,
// 1.5 ms for one wave; a collapsed filter's heavy siblings sit side by side, 64
// sources of ~2000 outputs in one wave, 0.7 ms).
constexpr int64_t kWaveFill = 4096;
constexpr int64_t kFillChunk = 4096;
constexpr int kMaxLongRuns = 65536;
constexpr unsigned kTailFill = 64;         // k_tail_single workgroups filling listed runs

struct DevStats {
    double total;            // normalise total (sum of w after update)
    double sumsq;            // sum of normalised w^2
    double n_eff;
    double u0;
    double best_w;
    double pose[3];
    int64_t best_index;      // local index of the estimate particle
    int32_t resampled;
    int32_t max_count;
    int32_t error_flags;
    uint32_t pad1;
    unsigned long long visited, candidates, hits, appends, written, ambiguous, resample_slots;
    unsigned long long words;    // candidate list entries (8 B: slot, record) written by k_candidates
    unsigned long long cow_pages;    // pages copied before their first write (shared)
    unsigned long long new_pages;    // fresh pages (appends, received particles)
    unsigned long long groups;       // page groups streamed by k_candidates
    double offset;           // global prefix of weights before this rank's first particle
    double t_local;          // sum of this rank's normalised weights (last local prefix)
    int32_t out_min, out_max;   // smallest / largest output index served by a local particle
    int32_t n_recv;          // particles received from other ranks by the resample
    int32_t collect_next;    // page_refs: some rank asked for a collective collection before the next scan
    unsigned long long reduce_amb;   // tree reductions: resample boundaries / the N_eff rule within
                                     // the rounding bound of the reference's summation order
    unsigned long long opened;       // pages whose mirrors k_candidates loaded
    unsigned long long ref_visits;   // landmarks the reference's first-match scan reads (j + 1 on a
                                     // match, the map size on an append)
    unsigned long long repeat_pages; // sharded: distinct pages sent that went to the same rank before
                                     // (since this rank's last collection; what a receiver-side page
                                     // cache could skip)
    unsigned long long loc_pages;    // page_refs: remote pages localised (free-list tail consumed)
    unsigned long long loc_recs;     //            records taken for them
    unsigned long long remote_rows;  //            a resample's outputs: row entries naming remote pages
    unsigned long long loc_rows;     //            row entries k_localize pointed at a local copy
    unsigned long long remote_pages; //            a resample's outputs: distinct remote pages their rows name
};

// Open-addressing set of tagged page ids (page_refs: k_localize's copies, the
// gather's distinct remote pages): keys epoch << 32 | id, a slot of an older epoch
// is free, so the table is never cleared.  Returns the slot and whether this call
// inserted the key (a claim), or -1 when the table is full.
__device__ inline int64_t ptable_insert(unsigned long long *key, int64_t cap, uint32_t epoch, uint32_t x,
                                        bool *claimed) {
    const unsigned long long want = ((unsigned long long)epoch << 32) | x;
    const uint64_t mask = (uint64_t)cap - 1u;
    uint64_t s = ((uint64_t)x * 0x9E3779B97F4A7C15ull >> 20) & mask;
    *claimed = false;
    for (int64_t probe = 0; probe < cap;) {
        const unsigned long long cur = __atomic_load_n(&key[s], __ATOMIC_RELAXED);
        if (cur == want) return (int64_t)s;
        if ((cur >> 32) != epoch) {
            if (atomicCAS(&key[s], cur, want) == cur) {
                *claimed = true;
                return (int64_t)s;
            }
            continue;                      // taken meanwhile: look again
        }
        s = (s + 1) & mask;
        ++probe;
    }
    return -1;
}

// numpy's np.sum over 8192-element buffers (fs2_exact.hip).  The recursion over a
// partial last chunk is fixed by the handle's particle count (np_tail_plan, host):
// its leaves in order, then its internal nodes in post-order, node nl + k = node
// a[k] + node b[k] (the last is the root).
constexpr int kNpChunk = 8192;
constexpr int kNpMaxLeaves = 256;
struct NpTailPlan {
    int32_t nl;                      // leaves (0: no partial chunk)
    int32_t off[kNpMaxLeaves], len[kNpMaxLeaves];
    int32_t a[kNpMaxLeaves], b[kNpMaxLeaves];
};

// Per-rank record all-gathered once per scan (and once more after a resample).
struct RankRecord {
    double sumsq;            // sum of normalised w^2 (local)
    double best_w;
    int64_t best_gidx;       // global index of the local first maximum
    double pose[3];
    double t_local;          // local normalised total (prefix end)
    int32_t max_count;
    int32_t want_collect;    // page_refs: this rank's pools run short (collective collection next scan)
};

constexpr int kMaxRanks = 16;

// ---- exact-order reductions across shards (fs2_exact.hip) ----
//
// Python's sum over the global particle order, split over G shards: each rank
// classifies its chain units against an estimate of the global prefix (its
// shard's offset from the all-gathered tree totals) and exports its chain as a
// list of fp64 adds ("ops": one per translation run, one per segment, one per
// term of a unit evaluated term by term) that is exact for its true entry value.
// Every rank folds all ranks' ops in shard order: the exact total, and the exact
// chain value at its own first element, from which it walks its own units.
constexpr int kChainOpsCap = 2046;
struct ShardOrder {
    int8_t r[kMaxRanks];     // rank holding shard q
};
struct ChainSummary {
    int32_t nops;            // ops of this rank (> kChainOpsCap: overflow, not folded)
    int32_t pad[3];
    double ops[kChainOpsCap];
};
static_assert(sizeof(ChainSummary) == 16384, "ChainSummary layout");

// numpy's np.sum(w'^2) over the global order: 8192-element chunks (the last one
// partial: NpTailPlan of n_global), the chunk sums added in order.  A chunk cut by
// a shard boundary is described by both ranks: the leaves each holds whole (their
// sums) and the raw elements of the leaf the boundary cuts (< 128).
constexpr int kShardChunks = 1024;          // whole chunks per rank (larger shards: tree mode)
struct NpEdge {
    int32_t chunk;           // global chunk index (-1: none)
    int32_t leaf0, nleaf;    // leaves [leaf0, leaf0 + nleaf) of the chunk's plan held whole
    int32_t cut;             // the leaf the boundary cuts (-1: the cut lies between leaves)
    int32_t rfrom, nraw;     // raw elements [rfrom, rfrom + nraw) of leaf `cut` (leaf-relative)
    int32_t pad[2];
    double leaf[128];        // sums of leaves leaf0 ..
    double raw[128];
};
struct RankRecordX {
    RankRecord base;
    int32_t nsums;           // chunks held whole, in order
    int32_t first_chunk;     // global index of the first of them
    int32_t pad[14];
    NpEdge head, tail;       // the chunk cut by this shard's first / last boundary
    double sums[kShardChunks];
};
static_assert(sizeof(RankRecordX) <= 16384, "RankRecordX fits an all-gather slot");

// A transfer to one rank (fs2_resample.hip, "packing"): K particle headers (64 B
// each), then one 32-bit entry per page-table row of each particle (S rows,
// padded to 64 B), then the U distinct pages those rows name, then C
// covariances.  Particles that descend from one ancestor share most pages, so U
// is far below S.  Entry = unique page index | kEntryOwned when the receiver may
// own the page (named once, by a particle filling one output).  A page travels
// compact (XferPage, 160 B): its slots' fp64 means and map indices; a slot's
// covariance only when it differs from the configured initial one (most
// landmarks keep it: appended with it, and only the observed ones change), the
// receiver rebuilding records and gate mirrors (mirror_of, a pure function of
// the record) bit for bit.
struct XferPage {
    uint32_t cbase;          // index of its first covariance among the transfer's
    uint8_t fill;            // slots in use
    uint8_t cmask;           // bit j: slot j's covariance follows in the covariance section
    uint16_t pad0;
    uint16_t slot[8];        // map index of each slot (the mirror's slot bits)
    uint64_t pad1;
    double2 xy[8];           // means
};
static_assert(sizeof(XferPage) == 160, "XferPage layout");
constexpr int kXferCovBytes = 32;
// Per destination, the words of xrow / xmat: particles K, rows S, distinct pages
// U, covariances C (all-gathered to every rank), and the run [i0, i1) of local
// particles that send there (k_pack_bounds; the dedup kernels' grid).
constexpr int kXrowWords = 6;
constexpr uint32_t kEntryOwned = 0x80000000u;
__host__ __device__ inline int64_t xfer_idx_off(int64_t K) { return K * 64; }
__host__ __device__ inline int64_t xfer_page_off(int64_t K, int64_t S) { return K * 64 + ((S * 4 + 63) / 64) * 64; }
__host__ __device__ inline int64_t xfer_cov_off(int64_t K, int64_t S, int64_t U) {
    return xfer_page_off(K, S) + U * (int64_t)sizeof(XferPage);
}
__host__ __device__ inline int64_t xfer_bytes(int64_t K, int64_t S, int64_t U, int64_t C) {
    return xfer_cov_off(K, S, U) + C * kXferCovBytes;
}

struct PackHeader {
    int64_t gsrc;            // global index of the source particle
    int32_t out_lo, out_hi;  // outputs it fills on the receiver (global, inclusive)
    int32_t cnt;
    int32_t soff;            // its first row entry within the transfer's entries
    double x, y, yaw, w;
    int64_t pad;
};

// What this rank sends to one destination (k_pack_bounds): the run [i0, i1) of
// local particles whose outputs may reach its shard [pa, pb), the exclusive
// counts of non-empty ranges / page-table rows before i0, and the transfer's
// particles / rows.
struct PackPlan {
    int64_t i0, i1;
    int64_t e0, c0;
    int64_t K, S;
    int64_t pa, pb;
};

// page_refs mode: a transfer is this preamble, the K headers, then every row of
// the particles as a descriptor naming the page where it lives (rank tag)
struct RefPreamble {
    float slb;               // the sender's lower bound on its mirrors' s (the receiver lowers its own)
    float org, cell, icell;  // the sender's summary grid: its boxes' codes are converted outwards
    int32_t rank;
    int32_t pad[11];
};
static_assert(sizeof(RefPreamble) == 64, "RefPreamble layout");
__host__ __device__ inline int64_t xfer_ref_bytes(int64_t K, int64_t S) { return 64 + K * 64 + S * 8; }

struct RecvPeer {
    const PackHeader *hdr;   // K headers
    const uint32_t *idx;     // row entries
    const XferPage *pages;   // U distinct pages
    const double2 *covs;     // their covariances that differ from the initial one (2 per)
    const XDesc *refs;       // page_refs mode: the rows' descriptors (tagged), with boxes
    const RefPreamble *pre;  // page_refs mode: the sender's preamble
    int32_t K;               // particles from this peer
    int32_t kbase;           // index of its first particle among all received
    int64_t U;               // distinct pages from this peer
    int64_t ubase;           // index of its first page among all received pages
};

// Page dedup of the outgoing transfers: an open-addressing table keyed by
// fill << 40 | (destination + 1) << 32 | page id (0: empty), whether more than
// one row entry names the key, its index among the destination's distinct
// pages, its covariance mask and the index of its first covariance; every
// outgoing row entry's table slot (| kEntryOwned when its particle fills one
// output), destination-major from ebase[p].
struct XferTable {
    unsigned long long *key;   // [cap]
    uint32_t *ref;             // [cap] 1: named by more than one row
    uint32_t *uidx;            // [cap]
    uint32_t *cmask;           // [cap] slots whose covariance is not the initial one
    uint32_t *cbase;           // [cap] index of the page's first covariance (destination's)
    uint32_t *eslot;           // [sum S] per row entry
    uint32_t *ulist;           // [sum S] destination p's distinct pages' slots from ebase[p]
    int64_t cap;               // power of two
    int32_t log2cap;
    int64_t ebase[kMaxRanks + 1];
    int64_t ubase[kMaxRanks + 1];   // exclusive prefix of U over destinations (k_pack_pages)
    int64_t i_lo, i_hi;      // local particles [i_lo, i_hi) hold every outgoing row
};

struct MeasPack {
    double d[kMaxM], b[kMaxM], ox[kMaxM], oy[kMaxM];
    float fx[kMaxM], fy[kMaxM];   // fp32 observed point for the gate mirror
    float fe[kMaxM];              // >= |ox - fx|, |oy - fy| (rounded up)
};

// Page references across ranks (sharded "page_refs" mode): a
// resample sends the page-table rows of the particles that change ranks, not
// their pages.  A descriptor whose page lives on rank q carries the tag q + 1 in
// bits kRefShift..30 (never the owned bit: a remote page is never written in
// place); local pages have tag 0 (local ids < 2^kRefShift in this mode).  Every
// rank maps every other rank's page pool, record pool and page marks (IPC), and
// localises a remote page -- copies it and its records into its own pools --
// before a kernel of the update pass could read it (k_localize: the pages the
// measurement bands leave open, and the row an append may write), so the update
// kernels only ever see local pages; the cold readers (export, clustering,
// collection marks) follow tags through PeerMaps.  A rank keeps the pages other
// ranks reference alive: collections are collective in this mode (every rank
// marks its remote references into the owners' marks before anyone sweeps).
constexpr int kRefShift = 27;
constexpr uint32_t kRefIdMask = (1u << kRefShift) - 1u;
constexpr int kRefMaxRanks = 15;
struct PeerMaps {
    char *pool[kMaxRanks];           // every rank's page pool (this rank's own included)
    char *recs[kMaxRanks];           // record pools
    uint8_t *mark[kMaxRanks];        // page marks (collection)
};
__host__ __device__ inline uint32_t ref_tag(uint32_t e) { return (e & 0x80000000u) ? 0u : (e >> kRefShift) & 15u; }
__host__ __device__ inline uint32_t ref_id(uint32_t e) { return (e & 0x80000000u) ? (e & 0x7fffffffu) : (e & kRefIdMask); }

// The maps of one particle buffer: page pool + page table.
struct MapRef {
    char *pool;              // page id p at pool + p * kPageBytes
    Desc *pt;                // [rows][n] page descriptors
    int64_t n;               // row stride (local particles)
    int32_t rows;            // rows allocated
    char *recs;              // record r at recs + r * kRecBytes
    SumFrame frame;          // summary grid of the row boxes
    float *slb;              // lower bound on every nonzero mirror s (lowered by every write)
    uint32_t *bbox;          // [nblocks][kBBoxRows] workgroup row boxes (null: rows > kBBoxRows)
    const PeerMaps *peers;   // page_refs mode: every rank's pools (device memory); null otherwise
};

// Free pages and records reserved for one launch: lane i's t-th new page is
// freel[base + t * n + i], its t-th new record rfreel[rbase + t * n + i]
// (coalesced across lanes; unused ones return at the next collection).
struct PageAlloc {
    const uint32_t *freel;
    int64_t base;
    const uint32_t *rfreel;
    int64_t rbase;
};

// The particle buffers of set b (A/B across resamples).  A scan enqueued before the
// host knows whether the previous one resampled (pipelined submit, fs2_api.hip)
// takes its buffers on the device: set (*gen & 1) is current, and k_tail_single
// bumps *gen when a resample made the other set current.
struct BufSet {
    double *x, *y, *yaw, *w;
    int32_t *cnt;
    Desc *pt;
    uint32_t *bbox;          // null when the maps outgrow the row boxes
};

struct UpdateParams {
    int64_t n;               // local particles
    int64_t blk0, blk1;      // workgroups [blk0, blk1) of kBlock particles in this launch
    int64_t nblk;            // workgroups of the whole pass (column stride of cpart)
    int64_t gidx0;           // global index of local particle 0
    double *x, *y, *yaw, *w;
    int32_t *cnt;
    MapRef map;
    const double *noise;     // injected normal draws (nullable -> Philox)
    uint64_t seed, scan;
    double sigma;            // std of the selected motion noise
    double rotation, translation;
    int32_t do_move;
    int32_t move_cand;       // do_move in k_candidates (the noise is final before it); k_update reads the moved pose
    int32_t m;               // measurements in this pass
    int32_t k0;              // first measurement index of this pass
    int32_t last_pass;
    double gate2;            // match iff 0 <= q < gate2  (sqrt(q) < gate)
    float gate2f;            // gate2 rounded up to fp32 (mirror test)
    int32_t filter;          // use the fp32 gate mirror
    PageAlloc alloc;         // up to m new pages per lane (copy-on-write, appends)
    uint64_t *cand;          // [kMaxCand][n] candidates, slot order: slot << 44 | position << 32 | record
    int32_t *ncand;          // [n] candidates found (> kMaxCand: list truncated)
    double R[4];
    double init_cov[4];
    int32_t *assoc;          // [M][n] or null
    double *wpart;           // [nblk] block partial sums of w (last pass)
    unsigned long long *cpart;   // [kNumCounters][nblk] block counters
    DevStats *stats;
    MeasPack meas;
    // k_candidates stores the slb its bands used; k_update's overflow scan tests page
    // boxes with it (exact: its pages' mirrors predate the pass), so it opens no page
    // those bands rejected -- none that k_localize left remote (page_refs mode)
    float *slb_pass;
    // one GPU: x .. cnt and map.pt / map.bbox come from sets[*gen & 1] (a scan may be
    // enqueued before the host knows whether the previous one resampled)
    const uint32_t *gen;     // null: the pointers above
    const BufSet *sets;
};

struct ReduceParams {
    int64_t n;               // local particles
    int64_t n_global;
    int64_t gidx0;
    double *w;
    const int32_t *cnt;
    const double *x, *y, *yaw;
    const double *wpart;     // update partials
    int32_t nwpart;
    unsigned long long *cpart;   // update counters [kNumCounters][nwpart]
    double *part_sq;         // normalise partials: sum w'^2
    double *part_best_w;
    int64_t *part_best_i;
    int32_t *part_maxcnt;
    int32_t nparts;
    double floor;
    int32_t sequential;      // one lane, the reference's orders
    int32_t exact;           // the reference's orders in parallel (fs2_exact.hip)
    double *np_part;         // exact: numpy chunk sums of w'^2 (k_finalize, beyond its LDS stage)
    int32_t n_np;            // their count
    double *np_leaf;         // exact: numpy's 128-element leaves of the full chunks (k_normalize)
    int32_t chunked;         // exact: k_normalize_chunks left np.sum's half-chunk terms in np_part
                             // and its partials (nparts = normalize_chunk_parts(n))
    double *part_pose;       // chunked: [3 nparts] pose of each partial's first maximum
    const NpTailPlan *np_tail;   // exact: the partial last chunk's tree (null: none)
    double flip_margin;      // tree mode: relative rounding bound for reduce_amb (0: off)
    double *part_w;          // [nparts] block sums of the normalised weights (k_normalize)
    int32_t t_from_parts;    // k_finalize: t_local = tree sum of part_w (sharded exact mode)
    int32_t want_collect;    // into this rank's record (page_refs mode)
    double *est_base;        // k_global_total: the tree prefix of the shards before this one (nullable)
    const double *u0_host;   // nullable: injected u0 value lives here (device copy)
    uint64_t seed, scan;
    DevStats *stats;
    RankRecord *rec;         // this rank's record (written by k_finalize)
    const RankRecord *recs;  // all ranks' records (== rec when world == 1)
    const double *totals;    // all ranks' weight totals (world > 1)
    int32_t world, rank;
    // the shard (slice of the global particle order) this rank holds and the
    // rank holding each shard: cross-rank sums run in shard order (DESIGN §5,
    // "output shards follow their sources")
    int32_t shard;
    int8_t rank_of[kMaxRanks];
    // one GPU: k_finalize publishes a scan whose rule did not fire (null: never)
    DevStats *pub_host;
    unsigned long long *pub_flag;
    unsigned long long pub_seq;
};

// The unit table of an evaluated chain (fs2_exact.hip k_chain_walk), as the
// resample's range kernel reads it to evaluate the running sum in place.
struct ChainView {
    const int32_t *uinfo;             // [nu] bit 0: listed (values in c), else binade (bit 1: identity)
    const unsigned long long *ugl;    // [nu] exclusive translation sum inside the unit's group
    const int32_t *uol;               // [nu] listed units of the group up to and including k
    const unsigned long long *bpd;    // [ng] exclusive translation sum before each group
    const int32_t *bpc;               // [ng] listed units before each group
    const int32_t *seql;              // listed units in order
    const double *sout;               // chain value after each listed unit
    const int32_t *uel;               // [nu] binade + 4096 of the last translation proper in the group up to k
    const int32_t *bpe;               // [ng] ... before each group (0: none)
};

// Resample of a shard of n particles / n outputs starting at global index a.
struct ResampleParams {
    int64_t n;
    int64_t N;               // global particles
    int64_t a;               // global index of local particle 0 (the sources)
    int64_t ao;              // global index of local output 0 (the shard kept; == a on one GPU)
    int32_t keep;            // shard whose outputs this rank keeps (not sent; == shard of a unless reassigned)
    int32_t ranges_mode;     // k_ranges: bit 0 store mlo / mhi (and count ties), bit 1 fill out_src
    double *w;               // normalised weights (current)
    double *c;               // local inclusive prefix [n]
    double *bsum;            // block sums (prefix)
    int32_t nblk;            // 1024-element blocks
    int32_t lazy;            // prefix kernels run only when the resample rule fired
    uint32_t *gen;           // one GPU: bumped by k_tail_single when the scan resampled (BufSet)
    // page_refs: the gather counts the distinct remote pages its outputs' rows name
    // (ptable_insert over the handle's page table, epoch tepoch) -- the room bound
    // of the localisations until the next resample
    unsigned long long *tkey;
    int64_t tcap;
    uint32_t tepoch;
    double flip_margin;      // tree prefix: relative rounding bound counted in reduce_amb (0: off)
    int32_t use_chain;       // running sum from the exact chain's units (c: serial units only)
    ChainView chain;
    int32_t *mlo, *mhi;      // [n] global output range served by each local particle
    int32_t *out_src;        // [n] source of each local output: >= 0 local, < 0 -(k+1) received
    int4 *runs;              // [kMaxLongRuns] (first, last local output, source): out_src pieces of the
                             // waves with more than kWaveFill outputs, filled by k_fill_runs (one
                             // GPU: by k_tail_single's other workgroups)
    uint32_t *runs_n;        // pieces listed (k_ranges); zeroed by the gather that follows
    const double *x, *y, *yaw;
    const int32_t *cnt;
    double *ox, *oy, *oyaw, *ow;
    int32_t *ocnt;
    MapRef map;              // current page table
    Desc *opt;               // next page table [rows][n]
    uint32_t *obbox;         // its workgroup row boxes (null: none)
    XDesc *rdesc;            // [nrecv][rows] descriptors (with boxes) of received particles' rows
    XDesc *udesc;            // [sum U] descriptors (with boxes) of the received distinct pages
    PageAlloc alloc;         // received page u -> page freel[base + u], its slot j ->
                             // record rfreel[rbase + 8 u + j]
    int32_t *rank_d;         // [n] non-empty ranges before i in its 1024-block
    int32_t *rank_e;         // [n] their page-table rows
    int64_t *iblk;           // [2 * nblk + 2] per-block totals -> exclusive offsets, grand totals
    double *part_best_w;
    int64_t *part_best_i;
    unsigned long long *part_slots;   // [blocks] slots of each gather workgroup's outputs
    DevStats *stats;
    RankRecord *rec;         // this rank's post-resample estimate record
    // packing for the other ranks (k_pack_plan / k_pack_bounds / k_pack_*)
    int32_t world, rank;
    PackPlan *plan;          // [world] per destination
    int64_t *xrow;           // [kXrowWords world] per destination (K, S, U, C, i0, i1)
    char *sbuf[kMaxRanks];   // per destination: the transfer (xfer_bytes)
    XferTable xt;
    uint32_t *sent_mask;     // [npool] bit p: the page went to rank p since the last collection (probe)
    double init_cov[4];      // the configured initial landmark covariance (compact transfers)
    // received particles
    int32_t npeers;
    RecvPeer peers[kMaxRanks];
    // page_refs mode: rows travel as tagged descriptors (k_pack_refs / k_unpack_refs),
    // an output owns a page only when its source fills one output in all (a page sent
    // by reference must not be written in place on the sender)
    int32_t refs;
    // one GPU: the post-resample estimate from the sources (k_ranges' partials), so
    // k_tail_single publishes the scan before the gather; the gather then runs on
    // a resample marker that outlives the publication's reset of the stats
    // (*go == go_seq, written by k_tail_single)
    int32_t est_early;
    unsigned long long *go;
    unsigned long long go_seq;
};

// A 64-term chain unit that is not one translation, as up to kChainSegs
// segments in order (fs2_exact.hip): meta = length (bits 0-6) | serial (bit 7) |
// (binade + 4096) << 8, 0 past the last segment; val = what the segment adds to
// the chain (a translation D * ulp, exact; a serial term), or for the chain's
// first unit the value after it.
constexpr int kChainSegs = 8;
constexpr int kChainGroup = 16;    // units per k_chain_units workgroup (1024 terms)
struct UnitRec {
    int32_t meta[kChainSegs];
    double val[kChainSegs];
};

// The reference's sequential sum / running sum of a[0..n) (a >= 0), in parallel
// and bit-exactly (fs2_exact.hip): s_0 = a_0, s_k = fl(s_{k-1} + a_k).
struct ChainParams {
    const double *a;
    int64_t n;
    const double *bsum;      // [nb] sums of 256-element blocks (any order: an estimate)
    int32_t nb;
    int32_t lazy;            // run only when stats->resampled
    const unsigned long long *cpart;   // non-null: fold these update counters [kNumCounters][ncpart]
    int32_t ncpart;
    DevStats *cstats;        // into these statistics (k_wsum's other job; total mode)
    int32_t *uinfo;          // [nu] per 64-term unit: (binade + 4096) << 2 for a translation (bit 1:
                             // identity, every term adds 0 wherever the chain is -- its binade is
                             // inherited, chain_elast); bit 0: listed: segments (UnitRec, count in
                             // bits 3-6), or bit 1: evaluated term by term (chain_unit)
    UnitRec *urec;           // [nu] segments of the units with uinfo bit 0
    double *sentry;          // [nu] chain value before each non-translation unit (by ordinal)
    long long *udelta;       // [nu] translation in ulps of the unit's binade
    unsigned long long *ugl; // [nu] exclusive scan of udelta inside each group of kChainGroup units
    int32_t *uol;            // [nu] listed units of the group up to and including k
    unsigned long long *bD;  // [ng] per group: translation sum
    int32_t *bC;             // [ng]            listed units
    uint32_t *bM;            // [ng]            listed-unit mask
    int32_t *uel;            // [nu] binade + 4096 of the last translation proper (not identity) in
                             // the group up to and including k (0: none)
    int32_t *bE;             // [ng] ... of the group; bpe: before each group (k_chain_walk)
    int32_t *bpe;
    unsigned long long *bpd; // [ng] exclusive scans of bD / bC (k_chain_walk)
    int32_t *bpc;
    int32_t *seql;           // [nu] serial units in order
    double *sout;            // [nu] chain value after each serial unit (by ordinal)
    double *c;               // nullable: the chain's values (prefix mode)
    double *total;           // nullable: the final value
    const DevStats *stats;
    double margin;           // relative bound on |estimate - chain| (doubled)
    // sharded ranks (exact mode): the chain's first element is local element 0 only
    // on the first shard; the estimates start from *est_base (the tree prefix of the
    // shards before); local unit 0 is always listed; k_chain_walk exports the ops
    // (ops_out) instead of walking, or walks from *s_entry
    int32_t chain_first;
    int32_t force_list0;
    const double *est_base;
    ChainSummary *ops_out;
    const double *s_entry;
    int32_t *uop;            // [nu] export: each listed unit's first op (by ordinal)
};
hipError_t launch_chain(const ChainParams &p, hipStream_t s, hipEvent_t e0 = nullptr);
// sharded exact mode: the local units and their ops (k_chain_units + k_chain_walk export)
hipError_t launch_chain_export(const ChainParams &p, hipStream_t s);
// fold every rank's ops in shard order (all: [world] summaries, by rank): the total
// into *total (nullable), the value before this rank's first element into *entry
// (nullable)
// (an overflowing summary writes nothing -- the tree estimates stay -- and counts
// one reduce_amb)
hipError_t launch_chain_fold(const ChainSummary *all, int32_t world, int32_t shard, const int8_t *rank_of,
                             double *total, double *entry, DevStats *stats, hipStream_t s);
// walk the local units from *p.s_entry (prefix mode: sentry / sout / c)
hipError_t launch_chain_walk_from(const ChainParams &p, hipStream_t s);
// numpy's Sigma w'^2 of this shard's chunks into *rx (sums of whole chunks, edges)
hipError_t launch_np_shard(const double *w, int64_t n, int64_t first, int64_t n_global, const NpTailPlan *gtail,
                           RankRecordX *rx, hipStream_t s);
// all ranks' RankRecordX (by rank): N_eff from the exact Sigma w'^2, decision,
// estimate, u0, tree offset (sharded exact mode's k_global_finalize)
hipError_t launch_global_finalize_x(const ReduceParams &p, const RankRecordX *all, const NpTailPlan *gtail,
                                    hipStream_t s);
// numpy np.sum(w ** 2): 8192-element chunks (k_normalize leaves, k_finalize trees);
// the partial last chunk's tree (NpTailPlan, fs2_chain.hpp) planned on the host
bool np_tail_plan(int64_t n, NpTailPlan *out);
int64_t np_sumsq_chunks(int64_t n);

// Launch of kernel k; with profiling events (e0: its start, e1: its end, either
// may be null) through hipExtLaunchKernel, which takes both from the dispatch
// itself: no marker packets between the kernels of a scan.
#define FS2_LAUNCH_EV(k, g, b, s, e0, e1, ...)                                   \
    do {                                                                         \
        if ((e0) || (e1)) hipExtLaunchKernelGGL(k, g, b, 0, s, e0, e1, 0, __VA_ARGS__); \
        else hipLaunchKernelGGL(k, g, b, 0, s, __VA_ARGS__);                     \
    } while (0)

// ---- launch wrappers (defined in fs2_*.hip; events: FS2_LAUNCH_EV) ----
hipError_t launch_candidates(const UpdateParams &p, hipStream_t s, hipEvent_t e0 = nullptr,
                             hipEvent_t e1 = nullptr);
hipError_t launch_update(const UpdateParams &p, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_wsum(const ReduceParams &p, hipStream_t s, hipEvent_t e0 = nullptr);
hipError_t launch_normalize(const ReduceParams &p, hipStream_t s);
// exact mode: normalise + numpy's Sigma w'^2 per 4096-weight half chunk (a partial
// last chunk whole) + per-workgroup partials, then k_finalize_chunked (one wave)
hipError_t launch_normalize_chunks(const ReduceParams &p, hipStream_t s);
int32_t normalize_chunk_parts(int64_t n);          // workgroups (partials) of launch_normalize_chunks
hipError_t launch_finalize_chunked(const ReduceParams &p, hipStream_t s);
hipError_t launch_global_total(const ReduceParams &p, hipStream_t s);
hipError_t launch_prefix(const ResampleParams &p, int sequential, hipStream_t s);
hipError_t launch_finalize(const ReduceParams &p, hipStream_t s);
hipError_t launch_global_finalize(const ReduceParams &p, hipStream_t s);
// resample, split where the sharded path needs the host (sizes of transfers)
hipError_t launch_resample_ranges(const ResampleParams &p, hipStream_t s, bool fill_runs = true);
hipError_t launch_pack_count(const ResampleParams &p, hipStream_t s);
// the distinct pages of every destination's rows (xt sized for sum S, key and
// ref zeroed by the caller), counted into xrow[6 p + 2], their covariances
// into xrow[6 p + 3]
hipError_t launch_pack_dedup(const ResampleParams &p, hipStream_t s);
// headers, row entries and pages into sbuf (sizes from the all-gathered xrow)
hipError_t launch_pack_write(const ResampleParams &p, hipStream_t s);
// page_refs mode: preamble, headers and tagged row descriptors into sbuf (transfer bases)
hipError_t launch_pack_refs(const ResampleParams &p, hipStream_t s);
// page_refs mode, before an update pass reads the maps: every remote page the
// measurement bands leave open (and the row an append may write) copied with its
// records into this rank's pools, from the free lists' tails (DevStats loc_*)
struct LocalizeParams {
    MapRef map;
    const int32_t *cnt;
    int64_t n;
    int64_t nblk;
    int32_t m;
    float gate2f;
    MeasPack meas;
    const uint32_t *freel;
    int64_t ftail;           // free pages [.., ftail): the k-th localised page is freel[ftail - 1 - k]
    const uint32_t *rfreel;
    int64_t rtail;           // records: the k-th localised page's slot j -> rfreel[rtail - 1 - (8 k + j)]
    int64_t pcap, rcap;      // pages / records the tails may give (past them: error_flags bit 3, the
                             // pass's update kernels exit at once, the scan fails)
    DevStats *stats;
    // one local copy per distinct remote page (round 5): open addressing over the
    // tagged page id, keys epoch << 32 | tagged id (a slot of an older epoch is
    // free, so the table is never cleared), the copy's page id alongside
    unsigned long long *key;
    uint32_t *val;
    int64_t cap;             // power of two, >= twice the row entries a pass may localise
    uint32_t epoch;          // this pass's (>= 1)
};
hipError_t launch_localize(const LocalizeParams &p, hipStream_t s);
// estimate: also this rank's post-resample record (k_estimate); one GPU leaves
// it to launch_tail_single
hipError_t launch_resample_apply(const ResampleParams &p, bool estimate, hipStream_t s);
hipError_t launch_global_best(const ReduceParams &p, hipStream_t s);
// End of a scan: the scan's DevStats into host memory (mapped, coherent), then
// *flag = seq (system scope, after the stats), and the device copy zeroed for
// the next scan.  The host spins on the flag instead of a stream sync.
hipError_t launch_publish(DevStats *stats, DevStats *host_stats, unsigned long long *host_flag,
                          unsigned long long seq, hipStream_t s, hipEvent_t e1 = nullptr);
// Sharded ranks, mid-scan: DevStats (decision, max count) and nx words of xmat
// into host (coherent, mapped), then *flag = seq.
hipError_t launch_post(const DevStats *stats, const int64_t *xmat, int32_t nx, char *host,
                       unsigned long long *host_flag, unsigned long long seq, hipStream_t s);
// One GPU, when the resample fired: k_estimate + k_global_best + k_publish (a
// scan whose rule did not fire was published by k_finalize, ReduceParams.pub_*).
hipError_t launch_tail_single(const ResampleParams &r, const ReduceParams &p, DevStats *host_stats,
                              unsigned long long *host_flag, unsigned long long seq, hipStream_t s,
                              hipEvent_t e1 = nullptr);

#ifdef FS2_PHASE_TIMING
hipError_t debug_phase_times(unsigned long long out[8], int reset);
hipError_t debug_icp_phase_times(unsigned long long out[4], int reset);
hipError_t debug_chain_times(unsigned long long out[8], int reset);
hipError_t debug_fin_times(unsigned long long out[8], int reset);
hipError_t debug_tail_times_update(unsigned long long out[32], int reset);
hipError_t debug_tail_times_exact(unsigned long long out[32], int reset);
hipError_t debug_tail_times_resample(unsigned long long out[32], int reset);
#endif
// particle p (of count) row k takes the reserved page alloc.base + k * count + p, its
// slot j record alloc.rbase + j * count + p (row-major: a wave's row is contiguous)
// (ext: atomicMax of the float bits of the largest finite |x|, |y| imported; slb
// lowered to the smallest nonzero mirror s)
// perm (nullable): maps of exactly perm_len slots are laid out with slot perm[j]
// at position j (a spatial order: compact page boxes); others in slot order
hipError_t launch_import(const double *stage, const int32_t *cnt_stage, int64_t first,
                         int64_t count, int32_t lm_cap, MapRef map, PageAlloc alloc,
                         int32_t rows_each, int32_t *cnt, uint32_t *ext, const int32_t *perm,
                         int32_t perm_len, hipStream_t s);
// workgroup row boxes of every particle's map, from its pages' mirrors (no-op without bbox)
hipError_t launch_bbox_build(MapRef map, const int32_t *cnt, hipStream_t s);
hipError_t launch_export(double *stage, int64_t first, int64_t count, int32_t lm_cap,
                         MapRef map, const int32_t *cnt, hipStream_t s);
hipError_t launch_fill(double *p, double v, int64_t n, hipStream_t s);
hipError_t launch_iota(uint32_t *p, int64_t n, hipStream_t s);
hipError_t launch_iota_from(uint32_t *p, uint32_t v0, int64_t n, hipStream_t s);   // p[e] = v0 + e

// page pool collection (fs2_pages.hip): mark the pages referenced by the n maps
// of `map`, then list every unmarked page of [0, npool) in freel; nfree_dev
// receives the count.
hipError_t launch_collect(MapRef map, const int32_t *cnt, int64_t npool, uint8_t *mark,
                          uint8_t epoch, int64_t *bcnt, uint32_t *freel, int64_t *nfree_dev,
                          hipStream_t s);
// the two halves of launch_collect for a collective collection (page_refs mode:
// every rank marks, a barrier, every rank sweeps); epochs: every rank's epoch
hipError_t launch_collect_mark(MapRef map, const int32_t *cnt, uint8_t *mark, uint8_t epoch, const uint8_t *epochs,
                               hipStream_t s);
hipError_t launch_collect_sweep(int64_t npool, uint8_t *mark, uint8_t epoch, int64_t *bcnt, uint32_t *freel,
                                int64_t *nfree_dev, hipStream_t s);
// after launch_collect with the same (mark, epoch): mark every record a live page
// refers to, then list every unmarked record of [0, nrecs) in rfreel
hipError_t launch_collect_records(const char *pool, int64_t npool, const uint8_t *mark, uint8_t epoch,
                                  int64_t nrecs, uint8_t *rmark, uint8_t repoch, int64_t *rbcnt,
                                  uint32_t *rfreel, int64_t *rnfree_dev, hipStream_t s);
int64_t collect_blocks(int64_t npool);

// known-landmark clustering (fs2_cluster.hip).  status: 0 ok, 1 non-finite input,
// 2 coordinate span too large.
hipError_t cluster_points(const double2 *pts, int64_t n, double eps, int64_t min_samples, double *centres_out,
                          int64_t centres_cap, int64_t *nclusters, int32_t *labels_out, int32_t *status,
                          hipStream_t s);
hipError_t gather_map_points(MapRef map, const int32_t *cnt, int64_t n, double2 **pts_out, int64_t *npts,
                             hipStream_t s);

// test hooks of the device generator (fs2_device.hpp): raw Philox4x32-10 blocks
// (counter c[4 i..], key k[2 i..]) and the motion sample's normals of (seed, stream)
// at indices first .. first + n - 1
hipError_t launch_debug_philox(int64_t n, const uint32_t *ctr, const uint32_t *key, uint32_t *out, hipStream_t s);
hipError_t launch_debug_normals(uint64_t seed, uint64_t stream, uint64_t first, int64_t n, double *out,
                                hipStream_t s);

// numpy's legacy RandomState on the device (fs2_mtrng.hip): results of one draw,
// and the attempts whose log the host recomputes with libm
struct MtMeta {
    int64_t accepted;        // accepted polar attempts among those evaluated
    int64_t last_attempt;    // index of the last attempt the draw consumed
    double gauss;            // cached second value after the draw (has_gauss)
    int32_t has_gauss;
    int32_t amb_n;           // attempts listed in MtAmb (may exceed the capacity)
    // numpy's state after the normals and after u0 too (k_mt_final)
    int64_t E;               // stream index of the first word not consumed by the normals
    int32_t pos_after, pos_after_u0;
    uint32_t w_u0[2];        // raw words E, E + 1 (u0)
    uint32_t key_after[624], key_after_u0[624];
};
struct MtAmb {
    double r2, x1, x2;
    int64_t rank;            // among the accepted attempts: outputs h0 + 2 rank, + 1
};
// raw stream words R[begin, end) from R[begin - 624, begin) (one wave)
hipError_t launch_mt_words(uint32_t *R, int64_t begin, int64_t end, hipStream_t s);
// N normals legacy_normal(0, sigma) from A attempts at R[pos0 ..] (P pairs needed,
// h0: gauss0 first), this rank's slice [first, first + n_local) into out
// (the input key is block b_in of R: R[624 b_in + pos] is word pos0)
hipError_t launch_mt_draw(const uint32_t *R, int64_t pos0, int64_t b_in, int64_t A, int64_t P, int64_t N, int32_t h0,
                          double gauss0, double sigma, int64_t first, int64_t n_local, double *out,
                          int32_t *boff, MtMeta *meta, MtAmb *amb, int32_t amb_cap, double *tab, int32_t tab_ready,
                          MtMeta *meta_host, hipStream_t s);   // tab: [2][97] log table, made here unless tab_ready
hipError_t launch_mt_patch(double *out, const int64_t *idx, const double *val, int64_t n, hipStream_t s);
// jump-ahead (fs2_mtrng.hip): G regions of J words made in parallel (J >= 2 x 20561,
// G <= kMtMaxGen); g: the polynomials of mt_jump_polys(J, G) ([G - 1][mt_poly_words()]);
// win: [G - 1][624] scratch.  R[0, 624) is the key; R[624, total) made.
constexpr int kMtMaxGen = 16;
hipError_t launch_mt_words_parallel(uint32_t *R, int64_t total, const uint64_t *g, int pw, int G, int64_t J,
                                    uint32_t *win, hipStream_t s);
bool mt_jump_polys(uint64_t J, int G, std::vector<uint64_t> &out);
int mt_poly_words();
bool mt_jump_host(const uint32_t key[624], uint64_t J, uint32_t out[624]);
hipError_t launch_mt_debug_log(const double *x, int64_t n, double *out, int32_t *amb, hipStream_t s);

hipError_t launch_icp(int32_t B, int32_t P, const double *src, const double *tgt,
                      int32_t n_tgt, int32_t max_iter, double thr, double *R, double *t,
                      int32_t *iters, hipStream_t s);
hipError_t launch_best_fit(const double *src, const double *tgt, int32_t n, double *Rt,
                           hipStream_t s);
hipError_t launch_line_filter(const double *in, int32_t n, const double *taps, int32_t r,
                              double *out, hipStream_t s);
hipError_t launch_mahalanobis(const double *a, const double *b, const double *cov, int32_t K,
                              double *out, int32_t *singular, hipStream_t s);
hipError_t launch_associate(const double *obs, const double *lm, int32_t L, double gate2,
                            int32_t *out, hipStream_t s);

}  // namespace fs2
