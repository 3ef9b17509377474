// fs2_api.hip -- C ABI of libfs2.so (include/fs2.h): handle, HBM state, the
// per-scan launch sequence of the FastSLAM 2.0 update, state import/export and
// the stateless ICP / LineFilter / association helpers.
#include <hip/hip_runtime.h>

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/fs2.h"
#include "fs2_comm.hpp"
#include "fs2_frontend.hpp"
#include "fs2_kernels.hpp"
#include "fs2_mtrng.hpp"
#include "fs2_plan.hpp"

using namespace fs2;
static_assert(kMaxRanks <= fs2comm::kShmMaxRanks, "shm transport rank table");

namespace {

thread_local std::string g_last_error;

int set_err(std::string *dst, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    if (dst) *dst = buf;
    return code;
}

#define HIP_TRY(h, expr)                                                                       \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return set_err((h) ? &(h)->err : nullptr,                                          \
                           e_ == hipErrorOutOfMemory ? FS2_ERR_OOM : FS2_ERR_HIP,              \
                           "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,    \
                           __LINE__);                                                          \
    } while (0)

// Smallest q >= 0 with sqrt(q) >= gate: sqrt(q) < gate  <=>  q < gate2.
double gate_to_q(double gate) {
    if (!(gate > 0.0)) return 0.0;          // never matches (q >= 0 && q < 0)
    if (std::isinf(gate)) return INFINITY;
    double q = gate * gate;
    while (q > 0.0 && std::sqrt(std::nextafter(q, 0.0)) >= gate) q = std::nextafter(q, 0.0);
    while (std::sqrt(q) < gate) q = std::nextafter(q, INFINITY);
    return q;
}

// Profiling: six events per scan, taken by the dispatches themselves
// (hipExtLaunchKernel, FS2_LAUNCH_EV): 0 start of the update pass, 1 end of
// k_candidates, 4 start of k_update, 2 end of the update pass, 5 start of the
// reduction (k_wsum), 3 end of the publication.  Each profiled scan takes the
// next set of a pool and its times are read only by fs2_get_profile (or when the
// pool is used up), so no event query sits in the scan loop and no marker packet
// between kernels.
struct ProfScan {
    DevStats st{};
    int passes = 0;
    int m = 0;
    uint64_t fixed_bytes = 0;
};
constexpr int kProfSets = 128;
struct ProfEvents {
    hipEvent_t e[kProfSets][6] = {};
    ProfScan scan[kProfSets];
    bool ok = false;
    int used = 0;            // sets holding a scan not yet folded
};

// Device memory that grows in place: a virtual range reserved
// once, physical chunks mapped at its end as the pool grows (hipMemCreate /
// hipMemMap / hipMemSetAccess), so a growth copies nothing and the pool's address
// never changes.  Handles whose pools are shared with other ranks by IPC
// (page_refs) use plain allocations instead.
struct GrowMem {
    char *base = nullptr;
    size_t reserved = 0, mapped = 0, gran = 0;
    int device = 0;
    bool shareable = false;        // chunks exportable as POSIX file descriptors (page_refs between processes)
    std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> chunks;
};
static hipMemAllocationProp gm_prop(int device, bool shareable = false) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    if (shareable) prop.requestedHandleTypes = hipMemHandleTypePosixFileDescriptor;
    return prop;
}
// (a failure is reported once: the runtime's last error is cleared, so the
// caller's fallback launches do not inherit it)
static hipError_t gm_fail(hipError_t e) {
    (void)hipGetLastError();
    return e;
}
// Reserves room for `bytes` with headroom (half again, at least 64 MiB): modest,
// because the reservation is address space the process's other HIP runtimes
// (PyTorch's) may need; a growth beyond it moves the mapping, not the data.
static bool gm_init(GrowMem &g, int device, size_t bytes, bool shareable) {
    hipMemAllocationProp prop = gm_prop(device);
    size_t gran = 0;
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) != hipSuccess || !gran) {
        gm_fail(hipSuccess);
        return false;
    }
    const size_t want = bytes + std::max<size_t>(bytes / 2, size_t(64) << 20);
    const size_t r = (want + gran - 1) / gran * gran;
    void *p = nullptr;
    if (hipMemAddressReserve(&p, r, 0, nullptr, 0) != hipSuccess || !p) {
        gm_fail(hipSuccess);
        return false;
    }
    g.base = static_cast<char *>(p);
    g.reserved = r;
    g.gran = gran;
    g.device = device;
    g.shareable = shareable;
    return true;
}
static hipError_t gm_access(GrowMem &g, char *base, size_t bytes) {
    // access over everything mapped: setting it on the new chunk alone fails now
    // and then on ROCm 7.2 (scripts/vmm_probe.hip, profiles/r04_vmm_probe.txt)
    hipMemAccessDesc ad{};
    ad.location = gm_prop(g.device).location;
    ad.flags = hipMemAccessFlagsProtReadWrite;
    return hipMemSetAccess(base, bytes, &ad, 1);
}
// A larger reservation with the same physical chunks mapped at the same offsets
// (no data moves; the base changes: the caller drained the stream).
static hipError_t gm_relocate(GrowMem &g, size_t need) {
    const size_t want = std::max(need + need / 2, 2 * g.reserved);
    const size_t r = (want + g.gran - 1) / g.gran * g.gran;
    void *p = nullptr;
    hipError_t e = hipMemAddressReserve(&p, r, 0, nullptr, 0);
    if (e != hipSuccess || !p) return gm_fail(e != hipSuccess ? e : hipErrorOutOfMemory);
    char *nb = static_cast<char *>(p);
    size_t off = 0;
    for (auto &c : g.chunks) {
        e = hipMemMap(nb + off, c.second, 0, c.first, 0);
        if (e != hipSuccess) break;
        off += c.second;
    }
    if (e == hipSuccess && off > 0) e = gm_access(g, nb, off);
    if (e != hipSuccess) {
        size_t o = 0;
        for (auto &c : g.chunks) {
            if (o >= off) break;
            hipMemUnmap(nb + o, c.second);
            o += c.second;
        }
        hipMemAddressFree(nb, r);
        return gm_fail(e);
    }
    off = 0;
    for (auto &c : g.chunks) {
        hipMemUnmap(g.base + off, c.second);
        off += c.second;
    }
    hipMemAddressFree(g.base, g.reserved);
    g.base = nb;
    g.reserved = r;
    return hipSuccess;
}
// Physical chunks of closed handles, kept for the next handles' growth (process-
// wide).  A set of handles closed and a new set created in the same process: a
// large hipMemCreate of the new set waited 4.3 s (the round-4 driver bench's
// 2.9 s scan; profiles/r05_vmm_growth_trace.txt places it in hipMemCreate itself,
// ~5 us otherwise) even with the device drained before the release -- the driver
// is still reclaiming the tens of GB the closed handles released.  So pools grow
// in chunks of power-of-two sizes (kChunkMax, or the remainder rounded up), kept
// here on close and taken back by any later growth that needs a chunk of that size:
// no new physical memory, nothing for the driver to reclaim.  FS2_VMM_CACHE_MB caps
// what is kept (read at every close; default 0: nothing is kept, a closed handle's
// memory goes back to the device for PyTorch or any other allocator in the process
// -- a caller that closes and re-creates large handles opts in, as bench.py does);
// fs2_release_cached_memory() and an allocation that runs out of device memory
// release it.
constexpr size_t kChunkMax = size_t(256) << 20;
constexpr size_t kGuardBytes = size_t(64) << 10;     // FS2_GUARD: pattern after each buffer
constexpr int kGuardByte = 0xa5;
static size_t chunk_size(size_t remaining, size_t gran) {
    if (remaining >= kChunkMax) return kChunkMax;
    size_t c = gran;
    while (c < remaining) c <<= 1;
    return c;
}
struct ChunkCache {
    std::mutex mu;
    struct Chunk {
        int dev;
        bool shareable;
        size_t bytes;
        hipMemGenericAllocationHandle_t hd;
    };
    std::vector<Chunk> chunks;
    size_t bytes = 0;
    size_t cap() const {
        const char *e = std::getenv("FS2_VMM_CACHE_MB");
        return (e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)0) << 20;
    }
    bool put(const Chunk &c) {
        std::lock_guard<std::mutex> lk(mu);
        if (bytes + c.bytes > cap()) return false;
        chunks.push_back(c);
        bytes += c.bytes;
        return true;
    }
    bool take(int dev, bool shareable, size_t b, hipMemGenericAllocationHandle_t *hd) {
        std::lock_guard<std::mutex> lk(mu);
        for (size_t k = chunks.size(); k-- > 0;) {
            const Chunk &c = chunks[k];
            if (c.dev != dev || c.shareable != shareable || c.bytes != b) continue;
            *hd = c.hd;
            bytes -= b;
            chunks.erase(chunks.begin() + (ptrdiff_t)k);
            return true;
        }
        return false;
    }
    size_t release() {
        std::lock_guard<std::mutex> lk(mu);
        size_t n = 0;
        for (auto &c : chunks) {
            (void)hipMemRelease(c.hd);
            n += c.bytes;
        }
        chunks.clear();
        bytes = 0;
        return n;
    }
};
ChunkCache g_chunks;

// Test hook (fs2_debug_vm_fail_after_relocate): the next growth that had to move
// its mapping fails right after the move, as a failing hipMemCreate / hipMemMap /
// hipMemSetAccess would; the callers then fall back to allocate and copy from the
// moved mapping (g.base), never from the pointer they held before the growth.
std::atomic<int> g_vm_fail_after_relocate{0};
// FS2_TRACE: the host time of each step of a growth (where a slow growth waits)
struct GmStep {
    const char *what;
    size_t bytes;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~GmStep() {
        static const bool on = std::getenv("FS2_TRACE") != nullptr;
        if (!on) return;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::fprintf(stderr, "[fs2 vmm] %s %zu MiB %.3f ms\n", what, bytes >> 20, ms);
    }
};
// (a chunk that cannot be used after all goes back to the cache, or is released)
static void gm_drop(const GrowMem &g, size_t b, hipMemGenericAllocationHandle_t hd) {
    if (!g_chunks.put(ChunkCache::Chunk{g.device, g.shareable, b, hd})) (void)hipMemRelease(hd);
}
static hipError_t gm_grow(GrowMem &g, size_t bytes) {
    const size_t need = (bytes + g.gran - 1) / g.gran * g.gran;
    if (need <= g.mapped) return hipSuccess;
    // the chunks this growth maps, largest first (a last one rounded up to a power of two)
    std::vector<size_t> plan;
    size_t want = g.mapped;
    while (want < need) {
        plan.push_back(chunk_size(need - want, g.gran));
        want += plan.back();
    }
    if (want > g.reserved) {
        GmStep st{"relocate", want};
        const hipError_t e = gm_relocate(g, want);
        if (e != hipSuccess) return e;
        if (g_vm_fail_after_relocate.exchange(0)) return gm_fail(hipErrorOutOfMemory);
    }
    hipMemAllocationProp prop = gm_prop(g.device, g.shareable);
    const size_t mapped0 = g.mapped, nchunks0 = g.chunks.size();
    hipError_t e = hipSuccess;
    int cached = 0;
    {
        GmStep st{"chunks", want - mapped0};
        for (size_t b : plan) {
            hipMemGenericAllocationHandle_t hd{};
            if (g_chunks.take(g.device, g.shareable, b, &hd)) {
                ++cached;
            } else {
                e = hipMemCreate(&hd, b, &prop, 0);
                if (e == hipErrorOutOfMemory && g_chunks.release() > 0) {   // the kept chunks make room
                    (void)hipGetLastError();
                    e = hipMemCreate(&hd, b, &prop, 0);
                }
                if (e != hipSuccess) break;
            }
            e = hipMemMap(g.base + g.mapped, b, 0, hd, 0);
            if (e != hipSuccess) {
                gm_drop(g, b, hd);
                break;
            }
            g.chunks.push_back({hd, b});
            g.mapped += b;
        }
    }
    if (e == hipSuccess) {
        GmStep st{"access", want};
        e = gm_access(g, g.base, want);
    }
    if (e != hipSuccess) {          // back to where it was: this growth's chunks unmapped, kept
        while (g.chunks.size() > nchunks0) {
            const auto c = g.chunks.back();
            g.chunks.pop_back();
            g.mapped -= c.second;
            (void)hipMemUnmap(g.base + g.mapped, c.second);
            gm_drop(g, c.second, c.first);
        }
        g.mapped = mapped0;
        return gm_fail(e);
    }
    if (cached && std::getenv("FS2_TRACE")) std::fprintf(stderr, "[fs2 vmm] %d of %zu chunks from closed handles\n", cached, plan.size());
    return hipSuccess;
}
// (the caller drained the device: fs2_destroy.  A release the runtime must defer
// because work is still in flight is what made the next handle's first growth wait
// seconds -- profiles/r04_g8_refs_growth_probe.txt)
static void gm_free(GrowMem &g) {
    GmStep st{"free", g.mapped};
    size_t off = g.mapped;
    for (auto it = g.chunks.rbegin(); it != g.chunks.rend(); ++it) {
        off -= it->second;
        hipMemUnmap(g.base + off, it->second);
        gm_drop(g, it->second, it->first);      // kept for the next handle's growth
    }
    g.chunks.clear();
    if (g.base) hipMemAddressFree(g.base, g.reserved);
    g = GrowMem{};
}

}  // namespace

// One draw's context, from its start (mt_begin) to its end (mt_end): a
// synchronous fs2_mt_draw runs both back to back on the handle's stream; a
// deferred one (fs2_mt_draw_deferred) runs mt_begin on the draw stream and
// leaves mt_end to the next scan's submit, between k_candidates (which does not
// read the motion draws) and k_update, so that the host's work on the draw --
// waiting for the counts, the listed logs, the patches -- overlaps the
// candidate pass instead of preceding the scan.
struct MtCtx {
    fs2_mt_state in;
    double sigma = 0.0;
    int64_t N = 0, P = 0, A = 0, amb_cap = 0, pos0 = 0, have = 0, total = 0;
    int h0 = 0;
    fs2_mt_state *after = nullptr, *after_u0 = nullptr;
    double *u0_out = nullptr;
};

struct fs2_handle {
    fs2_config cfg{};
    int64_t n_global = 0, n = 0, first = 0;
    hipStream_t stream = nullptr;
    int cur = 0;
    double *x[2] = {}, *y[2] = {}, *yaw[2] = {}, *w[2] = {};
    int32_t *cnt[2] = {};
    // landmark pages (fs2_kernels.hpp): pool, page tables A/B, free list
    char *pool = nullptr;
    int64_t npool = 0;                     // pages in the pool
    GrowMem pool_vm, rpool_vm;             // in-place growth of the page / record pools (base null: hipMalloc)
    GrowMem mark_vm, freel_vm, rmark_vm, rfreel_vm;   // their marks and free lists, alike
    int64_t bcnt_cap = 0, rbcnt_cap = 0;   // sweep block counts allocated (collect_blocks)
    Desc *pt[2] = {};                      // [rows][n] page descriptors (A/B across resamples)
    uint32_t *bbox[2] = {};                // [nblocks][kBBoxRows] workgroup row boxes of pt[0] / pt[1]
    XDesc *rdesc = nullptr;                // received particles' rows [n_recv][rows] (with boxes)
    XDesc *udesc = nullptr;                // received distinct pages [u_recv] (with boxes)
    size_t udesc_cap = 0;
    // page dedup of the outgoing transfers (XferTable)
    unsigned long long *xt_key = nullptr;
    uint32_t *xt_ref = nullptr, *xt_uidx = nullptr, *xt_cmask = nullptr, *xt_cbase = nullptr;
    uint32_t *xt_eslot = nullptr, *xt_ulist = nullptr;
    int64_t xt_cap = 0, xt_ecap = 0;
    SumFrame frame{-127.0f, 1.0f, 1.0f};         // summary grid (fs2_kernels.hpp), grown by imports
    float ext_seen = 0.0f;                 // largest |x|, |y| imported so far
    float *slb = nullptr;                  // device: lower bound on every nonzero mirror s
    float *slb_pass = nullptr;             // device: slb at the start of the current update pass
    uint32_t *ext_dev = nullptr;           // device: import extent (float bits)
    size_t rdesc_cap = 0;
    int rows = 0;                          // page-table rows allocated
    uint32_t *freel = nullptr;             // free page ids [0, nfree)
    int64_t nfree = 0, cursor = 0;         // free pages listed / reserved since the last collection
    uint8_t *mark = nullptr;               // collection marks, one byte per page
    uint32_t *sent_mask = nullptr;         // sharded: per page, the ranks it went to since the last collection
    uint8_t epoch = 0;
    int64_t *bcnt = nullptr;               // sweep block counts -> offsets
    int64_t *nfree_dev = nullptr;
    uint64_t collections = 0;
    // slot records (fs2_kernels.hpp): pool, free list, marks (collected with the pages)
    char *rpool = nullptr;
    int64_t nrecs = 0;
    uint32_t *rfreel = nullptr;
    int64_t rnfree = 0, rcursor = 0;
    uint8_t *rmark = nullptr;
    uint8_t repoch = 0;
    int64_t *rbcnt = nullptr;
    int64_t *rnfree_dev = nullptr;
    int64_t u_recv = 0;                    // distinct pages received by the last resample
    int32_t *rank_d = nullptr, *rank_e = nullptr;
    int64_t *iblk = nullptr;
    int cap = 0, max_cap = kMaxSlots;
    double *wpart = nullptr, *part_sq = nullptr, *part_best_w = nullptr, *part_pose = nullptr;
    unsigned long long *cpart = nullptr;   // update-pass block counters [kNumCounters][nblocks]
    int64_t *part_best_i = nullptr;
    unsigned long long *part_slots = nullptr;   // gather: slots per output workgroup
    int32_t *part_maxcnt = nullptr;
    double *cbuf = nullptr, *bsum = nullptr;
    DevStats *stats_dev = nullptr;
    // mid-scan posts of sharded ranks (k_post): DevStats + transfer sizes, then the flag
    char *post_host = nullptr, *post = nullptr;       // host / device view of one coherent block
    unsigned long long *post_flag = nullptr, *post_flag_dev = nullptr;
    unsigned long long post_seq = 0;
    PackPlan *plan = nullptr;                       // [kMaxRanks] what goes to each rank
    // end-of-scan publication (k_publish): stats + sequence flag in coherent host memory
    DevStats *pub_stats = nullptr, *pub_stats_dev = nullptr;
    unsigned long long *pub_flag = nullptr, *pub_flag_dev = nullptr;
    unsigned long long pub_seq = 0;
    bool stats_clean = false;              // stats_dev is zero (k_publish ran last)
    double *noise_dev = nullptr, *noise_pin = nullptr, *u0_dev = nullptr, *u0_pin = nullptr;
    // numpy's legacy RandomState on the device (fs2_mt_draw): stream words, block
    // offsets, results, listed logs, host patches; the next scan uses its draws
    struct MtWork {
        // two word buffers: the draw reads raw[cur]; the next draw's words are made
        // ahead into raw[1 - cur] on `side` while the scan runs (the stream does not
        // depend on how many words a draw consumes)
        uint32_t *raw[2] = {};
        int64_t raw_cap[2] = {};
        int cur = 0;
        hipStream_t side = nullptr;
        hipEvent_t ev_words = nullptr, ev_pre = nullptr;
        bool pre_valid = false;
        uint32_t pre_key[2][624];          // the states the next draw may start from
        int32_t pre_spos[2];               // their pos
        int64_t pre_pos0[2];               // their first word in raw[1 - cur]
        int64_t pre_total = 0;             // words made ahead in raw[1 - cur]
        int32_t *boff = nullptr;
        int64_t boff_cap = 0;
        MtMeta *meta = nullptr, *meta_pin = nullptr;
        MtAmb *amb = nullptr, *amb_pin = nullptr;
        int64_t amb_cap = 0;
        uint32_t *words_pin = nullptr;     // [2 kMtN]: key in, state blocks out
        int64_t *pidx = nullptr, *pidx_pin = nullptr;
        double *pval = nullptr, *pval_pin = nullptr;
        int64_t patch_cap = 0, pval_cap = 0;
        double *tab = nullptr;             // [2][97] log table (device)
        // jump-ahead: G regions of J words made in parallel (J, G fixed per handle)
        int64_t jJ = 0;
        int jG = 0;                        // 0: not planned, 1: sequential
        uint64_t *jpoly = nullptr;         // [G - 1][mt_poly_words()]
        uint32_t *jwin = nullptr;          // [G - 1][624]
        bool tab_ready = false;
        bool armed = false;
        // a deferred draw (fs2_mt_draw_deferred), enqueued on dstream, ended by the next submit
        hipStream_t dstream = nullptr;
        hipEvent_t ev_in = nullptr, ev_noise = nullptr;
        bool deferred = false;
        MtCtx dc;
        // (round 5 began the next scan's draw speculatively when a scan completed;
        // measured neutral twice on the drop-in -- profiles/r05_dropin_ab.json -- and
        // removed in round 6: each draw is begun by its own fs2_mt_draw_deferred)
    } mt;
    int32_t *assoc_dev = nullptr;
    int64_t assoc_cap = 0;
    int32_t last_m = 0;
    uint64_t scan = 0;
    // a scan enqueued by fs2_iterate_submit, completed by fs2_iterate_wait
    struct Pending {
        bool on = false;
        unsigned long long seq = 0;
        bool prof = false;
        int passes = 0;
        int32_t m = 0;
        uint64_t fixed_bytes = 0;
    } pending;
    // Pipelined submit (fs2.h fs2_iterate_submit): scan s+1 submitted while scan s is
    // outstanding.  Its update pass is enqueued behind s's tail, taking its buffer set
    // on the device (BufSet, gen: the host does not know yet whether s resampled);
    // its own tail is enqueued when s is waited for (the host then knows the set).
    struct TailCtx {
        int32_t M = 0;
        int passes = 0;
        uint64_t fixed_bytes = 0;
        bool prof = false;
        int evset = 0;
        int32_t want_collect = 0;
        bool has_u0 = false;
        int par = 0;                       // parity of the scan's per-scan buffers (cpart, pins)
    };
    struct {                               // a scan completed early (a submit had to wait for it)
        bool on = false;
        int rc = FS2_OK;
        double pose[3] = {};
        fs2_iter_stats st{};
    } stash;
    uint32_t *gen_dev = nullptr;           // the current set is (gen & 1) == cur (one GPU)
    unsigned long long *go_dev = nullptr;  // one GPU: publication sequence of the last resampling scan (the gather's marker)
    BufSet *sets_dev = nullptr;            // [2]
    uint64_t submitted = 0;                // scans submitted (parity)
    int32_t cnt_upper = 0;
    double gate2 = 64.0;
    std::string err;
    bool profiling = false;
    int32_t prof_period = 1;               // profile every prof_period-th scan
    uint64_t prof_tick = 0;
    ProfEvents ev;
    fs2_profile prof{};
    // sharding (world_size > 1)
    fs2comm::Transport *tp = nullptr;
    RankRecord *rec = nullptr, *recs = nullptr;     // this rank's record / all ranks'
    double *totals = nullptr;                       // all ranks' weight totals
    int64_t *xrow = nullptr, *xmat = nullptr;       // transfer sizes (particles, rows, pages, covariances) per peer
    int32_t *mlo = nullptr, *mhi = nullptr, *out_src = nullptr;
    uint32_t *runs_n = nullptr;
    int4 *runs = nullptr;                           // k_ranges' long output runs (k_fill_runs)
    uint64_t *cand = nullptr;                       // [kMaxCand/4][n] candidate slots
    int32_t *ncand = nullptr;
    // the sharded resample's transfers: one send and one receive arena, each
    // destination's (source's) transfer at an aligned offset
    char *sarena = nullptr, *rarena = nullptr;
    size_t scap = 0, rcap = 0;
    int32_t n_recv = 0;                             // particles received by the last resample
    // which slice of the global particle order (shard) this rank holds, and the
    // rank holding each shard.  With equal shards a resample may hand a rank
    // another shard, the one its own sources fill most (exchange_particles):
    // `follow`.  first = shard_begin(shard).
    int32_t shard = 0;
    int8_t rank_of[kMaxRanks] = {};
    bool follow = false;
    uint64_t shard_moves = 0;                       // resamples that changed this rank's shard

    // exact-order reductions (fs2_exact.hip)
    int32_t *uinfo = nullptr, *uol = nullptr, *seql = nullptr, *bC = nullptr, *bpc = nullptr;
    uint32_t *bM = nullptr;
    int32_t *uel = nullptr, *bE = nullptr, *bpe = nullptr;
    long long *udelta = nullptr;
    unsigned long long *ugl = nullptr, *bD = nullptr, *bpd = nullptr;
    double *sout = nullptr, *part_w = nullptr, *np_part = nullptr, *np_leaf = nullptr, *sentry = nullptr;
    NpTailPlan *np_tail = nullptr;         // device: numpy's tree over the partial last chunk (null: none)
    UnitRec *urec = nullptr;
    // exact-order reductions across shards (sharded EXACT mode): this rank's chain
    // ops and all ranks', this rank's reduction record and all ranks', the tree
    // estimate of the chain before this shard, each listed unit's first op, and
    // numpy's plan of the global partial last chunk
    bool xsh_ok = false;
    // page_refs mode (fs2_kernels.hpp PeerMaps): every rank's pools mapped here; the
    // pages other ranks may reference stay alive through collective collections
    bool refs = false;                     // the mode is on
    bool refs_off = false;                 // turned off at the first scan (a rank could not map its peers)
    bool refuse_maps = false;              // test hook: this rank reports its peer mappings as failed
    bool room_check = false;               // page_refs: agree on pool room at the next scan (after a resample)
    bool refs_shared = false;              // pools mapped by the peers: they never move (no growth)
    bool vm_share = false;                 // page_refs between processes: pool chunks exportable (share_vm)
    uint32_t loc_epoch = 0;                // k_localize passes so far (its table's key epoch)
    bool refs_live = false;                // a resample has exchanged references (no local collection)
    uint64_t grows = 0;                    // collective pool growths
    uint64_t vm_fallbacks = 0;             // growths that left the reserved range (allocate and copy)
    // what a record collection could free at most: the free-list entries taken
    // since the last one minus the records appended since (the rest were unused
    // or replaced slots) -- a bound only while no particle was dropped (resample)
    // and no map replaced (import) since
    int64_t appends_since_rcollect = 0;
    bool rcollect_exact = true;            // (a new handle's pools hold no record yet)
    std::vector<uint8_t> imported;         // particles whose maps were imported before the first scan
    PeerMaps peers_host{};
    PeerMaps *peers_dev = nullptr;
    uint8_t *ep_dev = nullptr, *epochs_dev = nullptr;     // this rank's / every rank's collection epoch
    int64_t remote_rows = 0;               // upper bound on row entries naming remote pages (localisations)
    int64_t remote_pages = INT64_MAX;      // distinct remote pages the rows named after the last resample
    // what the update passes may still localise per scan: at most one copy per
    // distinct remote page and pass (k_localize), never more than the remote rows
    int64_t remote_bound() const { return std::min(remote_rows, remote_pages); }
    int32_t collect_next = 0;              // before the next scan: bit 0 a collective collection, bits 1 / 2
                                           // every rank grows its page / record pool (published)
    ChainSummary *dch_send = nullptr, *dch_recv = nullptr;
    RankRecordX *recx = nullptr, *recxs = nullptr;
    double *est_base = nullptr;
    int32_t *uop = nullptr;
    NpTailPlan *np_tail_g = nullptr;
    // profiling, sharded: a start / end event pair around each resample's exchange
    // (its device time: nothing else runs on the stream meanwhile), folded into
    // prof.exchange_ms by fs2_get_profile
    std::vector<std::pair<hipEvent_t, hipEvent_t>> xev;
    size_t xev_used = 0;
    // FS2_GUARD: the pattern after each buffer fs2_create made (fs2_debug_check_guards)
    struct Guard {
        char *at;
        const char *name;
    };
    std::vector<Guard> guards;

    MapRef map() const {
        return MapRef{pool, pt[cur], std::max<int64_t>(n, 1), rows, rpool, frame, slb, row_boxes(cur),
                      refs_shared ? peers_dev : nullptr};
    }
    // row boxes of buffer b, while the maps fit them (fs2_kernels.hpp)
    uint32_t *row_boxes(int b) const { return rows <= kBBoxRows ? bbox[b] : nullptr; }
    int64_t nblocks() const { return (n + kBlock - 1) / kBlock; }
    // the reduction order in force (FS2_REDUCE_*, AUTO resolved)
    int reduce() const {
        const int mode = cfg.reduce_mode;
        if (tp) {
            if (mode == FS2_REDUCE_SEQUENTIAL) return FS2_REDUCE_SEQUENTIAL;
            return (mode != FS2_REDUCE_PARALLEL && xsh_ok) ? FS2_REDUCE_EXACT : FS2_REDUCE_PARALLEL;
        }
        if (mode != FS2_REDUCE_AUTO) return mode;
        return n_global <= 4096 ? FS2_REDUCE_SEQUENTIAL : FS2_REDUCE_EXACT;
    }
    ChainParams chain(const double *a, const double *bsum, double *c, double *total, bool lazy) const {
        ChainParams p{};
        p.a = a;
        p.n = n;
        p.bsum = bsum;
        p.nb = (int32_t)nblocks();
        p.lazy = lazy ? 1 : 0;
        p.uinfo = uinfo;
        p.udelta = udelta;
        p.ugl = ugl;
        p.uol = uol;
        p.bD = bD;
        p.bC = bC;
        p.bM = bM;
        p.bpd = bpd;
        p.bpc = bpc;
        p.uel = uel;
        p.bE = bE;
        p.bpe = bpe;
        p.seql = seql;
        p.sout = sout;
        p.urec = urec;
        p.sentry = sentry;
        p.c = c;
        p.total = total;
        p.stats = stats_dev;
        // recursive summation of n terms >= 0: |chain - exact| <= gamma_n exact; the
        // block estimates add gamma_{n/256 + 30}; doubled, plus slack for the scaling
        // (sharded: the whole chain's length, the shards' estimates included)
        p.margin = std::ldexp(2.0 * (double)n_global + 8192.0, -53);
        p.chain_first = 1;
        return p;
    }
};

// A copy that touches the handle's memory, ordered on its (non-blocking) stream
// and complete on return.  A plain hipMemcpy between two device buffers may
// return before the copy ends and is not ordered with that stream, so a kernel
// or memset the handle enqueues next could overtake it (a chunked export read
// back zeros that way).
static hipError_t copy_sync(fs2_handle *h, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, h->stream);
    return e == hipSuccess ? hipStreamSynchronize(h->stream) : e;
}

// Host wall time of one transport call or mid-scan wait, into the profile.
struct CommTimer {
    fs2_handle *h;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit CommTimer(fs2_handle *hh) : h(hh) {}
    ~CommTimer();
};

CommTimer::~CommTimer() {
    if (!h->profiling) return;
    h->prof.comm_calls += 1;
    h->prof.comm_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Page-table rows for maps of up to need_slots slots (current buffer kept).
// Growth after the first sizing is geometric (a quarter more rows, at least 8):
// maps grow by about one slot per scan, and a growth drains the stream and
// reallocates both tables (~n * rows * 16 B), so row-by-row growth cost a
// realloc every few scans of a long run.  Rows past a map's count are never
// read (every kernel stops at ceil(cnt / 8)), so spare rows cost memory only.
// The sharded resample's receive-side row buffers (received particles' rows, the
// distinct received pages' descriptors), `bytes` each: every local output's whole
// row fits (a rank receives at most n particles, at most n * rows distinct pages),
// so a resample never allocates.  The stream is drained first.
static int recv_bufs(fs2_handle *h, size_t bytes) {
    if (bytes <= h->rdesc_cap && bytes <= h->udesc_cap) return FS2_OK;
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    for (int k = 0; k < 2; ++k) {
        XDesc *&p = k ? h->udesc : h->rdesc;
        size_t &cap = k ? h->udesc_cap : h->rdesc_cap;
        if (bytes <= cap) continue;
        hipFree(p);
        p = nullptr;
        cap = 0;
        HIP_TRY(h, hipMalloc(&p, bytes));
        cap = bytes;
    }
    return FS2_OK;
}

// The sharded resample's row-sized buffers for every row of the shard (a rank
// sends at most its n particles' rows, receives at most n outputs' rows): the page
// dedup table (twice the rows, a power of two) and the received rows / pages.
// At creation and with every row growth, so a resample never allocates them (the
// first resamples at G = 8 sent up to ~65 % of a rank's rows).
static int reserve_xfer_table(fs2_handle *h, int64_t cap, int64_t nrows, bool in_scan);
static int xfer_bufs(fs2_handle *h) {
    const int64_t S = std::max<int64_t>(h->n, 1) * h->rows;
    int lg = 10;
    while ((int64_t(1) << lg) < 2 * S && lg < 31) ++lg;
    const int rc = reserve_xfer_table(h, int64_t(1) << lg, S, false);
    return rc ? rc : recv_bufs(h, sizeof(XDesc) * (size_t)S);
}

// The two buffer sets on the device (BufSet, pipelined submit): at creation and
// whenever the page tables are reallocated (the stream is drained then).
static int sync_sets(fs2_handle *h) {
    if (!h->sets_dev) return FS2_OK;
    BufSet b[2];
    for (int k = 0; k < 2; ++k)
        b[k] = BufSet{h->x[k], h->y[k], h->yaw[k], h->w[k], h->cnt[k], h->pt[k], h->row_boxes(k)};
    HIP_TRY(h, copy_sync(h, h->sets_dev, b, sizeof b, hipMemcpyHostToDevice));
    return FS2_OK;
}

static int grow_rows(fs2_handle *h, int need_slots) {
    if (need_slots <= h->cap) return FS2_OK;
    if (need_slots > h->max_cap)
        return set_err(&h->err, FS2_ERR_CAPACITY, "map needs %d landmark slots, limit is %d",
                       need_slots, h->max_cap);
    int rows = (need_slots + kPageSlots - 1) / kPageSlots;
    if (h->rows > 0) {
        const int geo = h->rows + std::max(h->rows / 4, 8);
        // (spare rows never switch the workgroup row boxes off)
        const int lim = std::min(h->max_cap / kPageSlots, rows <= kBBoxRows ? kBBoxRows : INT_MAX);
        rows = std::max(rows, std::min(geo, lim));
    }
    const size_t row_bytes = sizeof(Desc) * (size_t)std::max<int64_t>(h->n, 1);
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    for (int b = 0; b < 2; ++b) {
        Desc *p = nullptr;
        HIP_TRY(h, hipMalloc(&p, row_bytes * rows));
        if (h->pt[b] && b == h->cur) HIP_TRY(h, copy_sync(h, p, h->pt[b], row_bytes * h->rows, hipMemcpyDeviceToDevice));
        hipFree(h->pt[b]);
        h->pt[b] = p;
    }
    h->rows = rows;
    h->cap = rows * kPageSlots;
    if (int rc = sync_sets(h)) return rc;
    // (sharded: the resample's row buffers follow, here where the stream is drained
    // anyway, not inside a later resample)
    if (h->rdesc) return xfer_bufs(h);
    return FS2_OK;
}

static int refs_short(fs2_handle *h, const char *what) {
    return set_err(&h->err, FS2_ERR_CAPACITY,
                   "page_refs mode: the %s pool ran short between collective collections (pools shared with "
                   "the other ranks cannot grow; size them with page_pool / record_pool)",
                   what);
}

// Collect the page pool: every page the current page table does not refer to
// becomes free (fs2_pages.hip); the reservation cursor restarts.  With
// `records`, the record pool is collected from the same marks as well.
static int collect_body(fs2_handle *h, bool records);
// (host wall time of collections and growths, fs2_profile)
struct PoolTimer {
    fs2_handle *h;
    bool grow;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~PoolTimer() {
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (grow) {
            h->prof.pool_grows += 1;
            h->prof.grow_ms += ms;
        } else {
            h->prof.pool_collections += 1;
            h->prof.collect_ms += ms;
        }
    }
};
static int collect(fs2_handle *h, bool records) {
    PoolTimer pt{h, false};
    return collect_body(h, records);
}
static int collect_body(fs2_handle *h, bool records) {
    hipStream_t s = h->stream;
    if (h->epoch == 255) {
        HIP_TRY(h, hipMemsetAsync(h->mark, 0, (size_t)h->npool, s));
        h->epoch = 0;
    }
    h->epoch += 1;
    HIP_TRY(h, launch_collect(h->map(), h->cnt[h->cur], h->npool, h->mark, h->epoch, h->bcnt, h->freel,
                              h->nfree_dev, s));
    HIP_TRY(h, hipMemcpyAsync(&h->nfree, h->nfree_dev, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    if (records && h->nrecs > 0) {
        if (h->repoch == 255) {
            HIP_TRY(h, hipMemsetAsync(h->rmark, 0, (size_t)h->nrecs, s));
            h->repoch = 0;
        }
        h->repoch += 1;
        HIP_TRY(h, launch_collect_records(h->pool, h->npool, h->mark, h->epoch, h->nrecs, h->rmark, h->repoch,
                                          h->rbcnt, h->rfreel, h->rnfree_dev, s));
        HIP_TRY(h, hipMemcpyAsync(&h->rnfree, h->rnfree_dev, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        h->rcursor = 0;
        h->appends_since_rcollect = 0;
        h->rcollect_exact = true;
    }
    // page ids are recycled from here on: the transfer probe starts over
    if (h->sent_mask) HIP_TRY(h, hipMemsetAsync(h->sent_mask, 0, sizeof(uint32_t) * (size_t)h->npool, s));
    HIP_TRY(h, hipStreamSynchronize(s));
    h->cursor = 0;
    h->collections += 1;
    return FS2_OK;
}

// page_refs mode, at the first scan (every rank takes part: the ranks of one
// process are created one after the other, so creation cannot wait for them):
// every rank's page pool, record pool and page marks, mapped here (IPC; the ranks
// of one process share pointers).  From now on the pools never move.
// FS2_TRACE=1: the sharing and collective steps of a rank on stderr (debugging)
static void trace(const fs2_handle *h, const char *what, int k = -1) {
    static const bool on = std::getenv("FS2_TRACE") != nullptr;
    if (!on) return;
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    std::fprintf(stderr, "[fs2 rank %d %.3f] %s %d\n", h->cfg.rank, t, what, k);
    std::fflush(stderr);
}

// A buffer the sharded resample had to reallocate inside a scan (fs2_profile.scan_allocs)
static void scan_alloc(fs2_handle *h, const char *what, size_t bytes) {
    h->prof.scan_allocs += 1;
    trace(h, what, (int)std::min<size_t>(bytes >> 20, INT32_MAX));
}

static int share_pools(fs2_handle *h, bool first) {
    const int G = h->cfg.world_size;
    hipStream_t s = h->stream;
    void *ptrs[kMaxRanks] = {};
    trace(h, "share_pools start", first ? 1 : 0);
    HIP_TRY(h, hipStreamSynchronize(s));
    // Every rank takes part in the three exchanges and in the agreement after
    // them whatever its own mappings did: if some rank cannot map its peers' pools
    // (no peer access between the devices), the mode turns off on every rank and
    // the resamples send pages, as they may (no reference has crossed yet).
    bool ok = true;
    std::string why;
    for (int what = 0; what < 3; ++what) {
        void *base = what == 0 ? (void *)h->pool : what == 1 ? (void *)h->rpool : (void *)h->mark;
        const GrowMem &vm = what == 0 ? h->pool_vm : what == 1 ? h->rpool_vm : h->mark_vm;
        CommTimer ct(h);
        std::string e;
        trace(h, "share", what);
        // pools grown in place go as their VMM chunks (every rank takes the same
        // path: vm_share is the same on every rank, and a pool that left its
        // reserved range fails the export, which the agreement below turns off)
        int src;
        if (h->vm_share) {
            std::vector<fs2comm::VmChunk> ch;
            if (vm.base == base)
                for (const auto &c : vm.chunks) ch.push_back({c.first, c.second});
            src = h->tp->share_vm(ch, base, h->cfg.device, ptrs, &e);
        } else {
            src = h->tp->share(base, ptrs, &e);
        }
        trace(h, "shared", src);
        if (src) {
            if (ok) why = e;
            ok = false;
            if (int rc = h->tp->status(&h->err)) return rc;     // the transport itself failed
            continue;
        }
        for (int q = 0; q < G; ++q) {
            if (what == 0) h->peers_host.pool[q] = (char *)ptrs[q];
            else if (what == 1) h->peers_host.recs[q] = (char *)ptrs[q];
            else h->peers_host.mark[q] = (uint8_t *)ptrs[q];
        }
    }
    if (h->refuse_maps && ok) {
        ok = false;
        why = "peer mappings refused (fs2_debug_refuse_peer_maps)";
    }
    uint8_t all[kMaxRanks] = {};
    trace(h, "agree", ok ? 1 : 0);
    HIP_TRY(h, hipMemsetAsync(h->ep_dev, ok ? 1 : 0, 1, s));
    {
        CommTimer ct(h);
        const int rc = h->tp->allgather(h->ep_dev, h->epochs_dev, 1, s, &h->err);
        if (rc) return rc;
    }
    HIP_TRY(h, hipMemcpyAsync(all, h->epochs_dev, (size_t)G, hipMemcpyDeviceToHost, s));
    HIP_TRY(h, hipStreamSynchronize(s));
    if (int rc = h->tp->status(&h->err)) return rc;
    bool every = true;
    for (int q = 0; q < G; ++q) every &= all[q] == 1;
    trace(h, "agreed", every ? 1 : 0);
    if (!every && !first)             // references have crossed: the grown pools must map
        return set_err(&h->err, FS2_ERR_COMM, "page_refs: mapping the grown pools failed (%s)",
                       ok ? "on another rank" : why.c_str());
    if (!every) {
        h->tp->unshare();
        h->refs = false;
        h->refs_off = true;
        return FS2_OK;
    }
    HIP_TRY(h, hipMemcpy(h->peers_dev, &h->peers_host, sizeof(PeerMaps), hipMemcpyHostToDevice));
    h->refs_shared = true;
    return FS2_OK;
}

// page_refs mode: a collection every rank runs at the same scan (the decision is
// in the all-gathered records, DevStats.collect_next).  Each rank's epoch reaches
// every rank (an all-gather, after each reset its marks), every rank marks its own
// pages and, in their owners' marks, the remote pages its rows name; a second
// all-gather is the barrier before anyone sweeps.  Records as in collect(): the
// remote-marked pages mark their records too.
static int collect_collective(fs2_handle *h) {
    trace(h, "collect_collective", (int)(h->nfree - h->cursor));
    hipStream_t s = h->stream;
    const int G = h->cfg.world_size;
    if (h->epoch == 255) {
        HIP_TRY(h, hipMemsetAsync(h->mark, 0, (size_t)h->npool, s));
        h->epoch = 0;
    }
    h->epoch += 1;
    HIP_TRY(h, hipMemsetAsync(h->ep_dev, h->epoch, 1, s));
    {
        CommTimer ct(h);
        const int rc = h->tp->allgather(h->ep_dev, h->epochs_dev, 1, s, &h->err);
        if (rc) return rc;
    }
    HIP_TRY(h, launch_collect_mark(h->map(), h->cnt[h->cur], h->mark, h->epoch, h->epochs_dev, s));
    {
        CommTimer ct(h);
        const int rc = h->tp->allgather(h->ep_dev, h->epochs_dev + kMaxRanks, 1, s, &h->err);
        if (rc) return rc;
    }
    HIP_TRY(h, launch_collect_sweep(h->npool, h->mark, h->epoch, h->bcnt, h->freel, h->nfree_dev, s));
    HIP_TRY(h, hipMemcpyAsync(&h->nfree, h->nfree_dev, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    if (h->nrecs > 0) {
        if (h->repoch == 255) {
            HIP_TRY(h, hipMemsetAsync(h->rmark, 0, (size_t)h->nrecs, s));
            h->repoch = 0;
        }
        h->repoch += 1;
        HIP_TRY(h, launch_collect_records(h->pool, h->npool, h->mark, h->epoch, h->nrecs, h->rmark, h->repoch,
                                          h->rbcnt, h->rfreel, h->rnfree_dev, s));
        HIP_TRY(h, hipMemcpyAsync(&h->rnfree, h->rnfree_dev, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(h, hipStreamSynchronize(s));
    if (int rc = h->tp->status(&h->err)) return rc;
    h->cursor = 0;
    h->rcursor = 0;
    if (h->nrecs > 0) {            // (as collect_body: the futile-collection bound starts over)
        h->appends_since_rcollect = 0;
        h->rcollect_exact = true;
    }
    h->collections += 1;
    (void)G;
    return FS2_OK;
}

// A pool's side array (marks, free list) grown to `bytes`, its first `keep` bytes
// kept: in place in a reserved range when the pools grow in place (reserved at
// the first growth), else allocated anew and copied.  *moved
// says which (a moved mark array restarts its epochs).
static int grow_side(fs2_handle *h, GrowMem &vm, void **ptr, size_t bytes, size_t keep, bool pools_in_place,
                     bool *moved) {
    *moved = false;
    // (a side array is small next to its pool -- 1 or 4 B per 48 B record -- so it
    // is mapped half again ahead and grows about every other pool growth)
    if (!vm.base && !*ptr && pools_in_place) gm_init(vm, h->cfg.device, 4 * bytes, h->vm_share);
    if (vm.base && (bytes <= vm.mapped || gm_grow(vm, std::max(bytes, vm.mapped + vm.mapped / 2)) == hipSuccess)) {
        *ptr = vm.base;
        return FS2_OK;
    }
    void *np = nullptr;
    HIP_TRY(h, hipMalloc(&np, bytes));
    // (a growth that failed after moving its mapping left the data at vm.base only)
    if (*ptr && keep) HIP_TRY(h, copy_sync(h, np, vm.base ? vm.base : *ptr, keep, hipMemcpyDeviceToDevice));
    if (vm.base) {
        gm_free(vm);
        h->vm_fallbacks += 1;
    } else {
        hipFree(*ptr);
    }
    *ptr = np;
    *moved = true;
    return FS2_OK;
}

// the sweep's per-block counts for `items` (capacity doubles: no free in a growth)
static int ensure_bcnt(fs2_handle *h, int64_t **b, int64_t *cap, int64_t items) {
    const int64_t need = collect_blocks(items);
    if (need <= *cap) return FS2_OK;
    hipFree(*b);
    *b = nullptr;
    *cap = 0;
    const int64_t c = std::max<int64_t>(need, 2 * need);
    HIP_TRY(h, hipMalloc(b, sizeof(int64_t) * (size_t)c));
    *cap = c;
    return FS2_OK;
}

// page_refs mode: every rank grows the pools some rank asked for (the flags are in
// the all-gathered records), together -- pools shared by IPC cannot grow in place:
// every rank unmaps the others' pools, a rendezvous, each reallocates its own
// (page and record ids keep their meaning), and the pools are shared anew.
static int grow_pool(fs2_handle *h, int64_t pages);
static int grow_recs(fs2_handle *h, int64_t n);
static int regrow_collective(fs2_handle *h, int64_t pages_to, int64_t recs_to) {
    trace(h, "regrow pages_to (M)", (int)(pages_to >> 20));
    trace(h, "regrow recs_to (M)", (int)(recs_to >> 20));
    hipStream_t s = h->stream;
    HIP_TRY(h, hipStreamSynchronize(s));
    h->tp->unshare();
    {
        CommTimer ct(h);
        const int rc = h->tp->allgather(h->ep_dev, h->epochs_dev + kMaxRanks, 1, s, &h->err);
        if (rc) return rc;
    }
    HIP_TRY(h, hipStreamSynchronize(s));
    h->refs_shared = false;
    int rc = FS2_OK;
    // (a target of 0: this rank's pool stays; it still takes part)
    if (pages_to > 0)
        rc = grow_pool(h, std::min<int64_t>(std::max(h->npool + h->npool / 2, pages_to), (int64_t)kRefIdMask - 1024));
    if (!rc && recs_to > 0)
        rc = grow_recs(h, std::min<int64_t>(std::max(h->nrecs + h->nrecs / 2, recs_to), (int64_t)kRecIdLimit));
    if (rc) return rc;
    h->grows += 1;
    return share_pools(h, false);
}

// Pool of `pages` pages (existing pages keep their ids), its free list and marks.
// The new pages are free: their ids join the free list after the entries already
// listed (no collection).  In place (GrowMem) when the handle's pools are not
// shared, else allocate and copy.
static int grow_pool(fs2_handle *h, int64_t pages) {
    if (pages <= h->npool) return FS2_OK;
    if (h->refs_shared) return refs_short(h, "page");
    PoolTimer pt{h, true};
    if (h->refs && pages > (int64_t)kRefIdMask)
        return set_err(&h->err, FS2_ERR_CAPACITY, "page_refs mode: %lld pages exceed the %u local page ids",
                       (long long)pages, kRefIdMask);
    if (pages > (int64_t)kIdMask)
        return set_err(&h->err, FS2_ERR_OOM, "page pool of %lld pages exceeds the id space", (long long)pages);
    hipStream_t s = h->stream;
    HIP_TRY(h, hipStreamSynchronize(s));
    // in place (VMM); page_refs between processes: chunks exportable as POSIX
    // descriptors (vm_share), mapped by the peers (Transport::share_vm)
    if (!h->pool) gm_init(h->pool_vm, h->cfg.device, (size_t)pages * kPageBytes, h->vm_share);
    if (h->pool_vm.base && gm_grow(h->pool_vm, (size_t)pages * kPageBytes) == hipSuccess) {
        h->pool = h->pool_vm.base;
    } else {
        // beyond the reservation, or the mapping failed: allocate and copy (the
        // reserved range is left for good)
        char *pool = nullptr;
        HIP_TRY(h, hipMalloc(&pool, (size_t)pages * kPageBytes));
        // (from the mapping itself: a growth that failed after moving it left the
        // pages at pool_vm.base, not at the h->pool held before)
        if (h->pool) HIP_TRY(h, copy_sync(h, pool, h->pool_vm.base ? h->pool_vm.base : h->pool,
                                          (size_t)h->npool * kPageBytes, hipMemcpyDeviceToDevice));
        if (h->pool_vm.base) {
            gm_free(h->pool_vm);
            h->vm_fallbacks += 1;
        } else {
            hipFree(h->pool);
        }
        h->pool = pool;
    }
    // marks and free list: in place with the pool (new marks zero, new ids after
    // the entries listed so far), else moved
    const bool vm = h->pool == h->pool_vm.base && h->pool_vm.base != nullptr;
    bool moved = false;
    int rc = grow_side(h, h->mark_vm, (void **)&h->mark, (size_t)pages, (size_t)h->npool, vm, &moved);
    if (rc) return rc;
    if (moved) {
        HIP_TRY(h, hipMemsetAsync(h->mark, 0, (size_t)pages, s));
        h->epoch = 0;
    } else {
        HIP_TRY(h, hipMemsetAsync(h->mark + h->npool, 0, (size_t)(pages - h->npool), s));
    }
    rc = grow_side(h, h->freel_vm, (void **)&h->freel, sizeof(uint32_t) * (size_t)pages,
                   sizeof(uint32_t) * (size_t)std::max<int64_t>(h->nfree, 0), vm, &moved);
    if (rc) return rc;
    HIP_TRY(h, launch_iota_from(h->freel + h->nfree, (uint32_t)h->npool, pages - h->npool, s));
    h->nfree += pages - h->npool;
    if (h->cfg.world_size > 1) {
        hipFree(h->sent_mask);
        h->sent_mask = nullptr;
        HIP_TRY(h, hipMalloc(&h->sent_mask, sizeof(uint32_t) * (size_t)pages));
        HIP_TRY(h, hipMemsetAsync(h->sent_mask, 0, sizeof(uint32_t) * (size_t)pages, s));
    }
    rc = ensure_bcnt(h, &h->bcnt, &h->bcnt_cap, pages);
    if (rc) return rc;
    h->npool = pages;
    return FS2_OK;
}

// Record pool of `n` records (existing records keep their ids), free list, marks:
// like grow_pool.
static int grow_recs(fs2_handle *h, int64_t n) {
    if (n <= h->nrecs) return FS2_OK;
    if (h->refs_shared) return refs_short(h, "record");
    PoolTimer pt{h, true};
    if (n > (int64_t)kRecIdLimit)
        return set_err(&h->err, FS2_ERR_OOM, "record pool of %lld records exceeds the 32-bit id space",
                       (long long)n);
    hipStream_t s = h->stream;
    HIP_TRY(h, hipStreamSynchronize(s));
    if (!h->rpool) gm_init(h->rpool_vm, h->cfg.device, (size_t)n * kRecBytes, h->vm_share);   // (as grow_pool)
    if (h->rpool_vm.base && gm_grow(h->rpool_vm, (size_t)n * kRecBytes) == hipSuccess) {
        h->rpool = h->rpool_vm.base;
    } else {
        char *rp = nullptr;
        HIP_TRY(h, hipMalloc(&rp, (size_t)n * kRecBytes));
        if (h->rpool) HIP_TRY(h, copy_sync(h, rp, h->rpool_vm.base ? h->rpool_vm.base : h->rpool,
                                           (size_t)h->nrecs * kRecBytes, hipMemcpyDeviceToDevice));
        if (h->rpool_vm.base) {
            gm_free(h->rpool_vm);
            h->vm_fallbacks += 1;
        } else {
            hipFree(h->rpool);
        }
        h->rpool = rp;
    }
    const bool vm = h->rpool == h->rpool_vm.base && h->rpool_vm.base != nullptr;
    bool moved = false;
    int rc = grow_side(h, h->rmark_vm, (void **)&h->rmark, (size_t)n, (size_t)h->nrecs, vm, &moved);
    if (rc) return rc;
    if (moved) {
        HIP_TRY(h, hipMemsetAsync(h->rmark, 0, (size_t)n, s));
        h->repoch = 0;
    } else {
        HIP_TRY(h, hipMemsetAsync(h->rmark + h->nrecs, 0, (size_t)(n - h->nrecs), s));
    }
    rc = grow_side(h, h->rfreel_vm, (void **)&h->rfreel, sizeof(uint32_t) * (size_t)n,
                   sizeof(uint32_t) * (size_t)std::max<int64_t>(h->rnfree, 0), vm, &moved);
    if (rc) return rc;
    HIP_TRY(h, launch_iota_from(h->rfreel + h->rnfree, (uint32_t)h->nrecs, n - h->nrecs, s));
    h->rnfree += n - h->nrecs;
    rc = ensure_bcnt(h, &h->rbcnt, &h->rbcnt_cap, n);
    if (rc) return rc;
    h->nrecs = n;
    return FS2_OK;
}

// Reserve `need` free pages (collecting, then growing the pool, when short);
// returns the reservation's first index into freel.  A launch that needs both
// reserves its records first: a record collection restarts the page cursor.
static int reserve_pages(fs2_handle *h, int64_t need, PageAlloc *out) {
    if (h->cursor + need > h->nfree) {
        if (h->refs_live) return refs_short(h, "page");
        int rc = collect(h, false);
        if (rc) return rc;
        if (need > h->nfree) {
            const int64_t live = h->npool - h->nfree;
            // by a quarter when the pool grows in place (cheap, no copy), else by half
            const int64_t step = h->pool_vm.base ? h->npool / 4 : h->npool / 2;
            rc = grow_pool(h, std::max(h->npool + step, live + 2 * need));
            if (rc) return rc;
        }
    }
    out->freel = h->freel;
    out->base = h->cursor;
    h->cursor += need;
    return FS2_OK;
}

static int reserve_recs(fs2_handle *h, int64_t need, PageAlloc *out) {
    if (h->rcursor + need > h->rnfree) {
        if (h->refs_live) return refs_short(h, "record");
        // a collection that cannot free enough is skipped: the pool grows at once
        // (the free list keeps its taken entries, the new ids follow it)
        const bool futile = h->rcollect_exact &&
                            (h->rnfree - h->rcursor) + (h->rcursor - h->appends_since_rcollect) < need;
        int rc = FS2_OK;
        if (!futile) {
            rc = collect(h, true);
            if (rc) return rc;
        }
        if (h->rcursor + need > h->rnfree) {
            const int64_t live = h->nrecs - (h->rnfree - h->rcursor);
            // by a quarter in place, else by half; clamped to the id space (grow_recs
            // fails beyond it)
            const int64_t step = h->rpool_vm.base ? h->nrecs / 4 : h->nrecs / 2;
            int64_t want = std::max(h->nrecs + step, live + 2 * need);
            if (want > (int64_t)kRecIdLimit) want = std::max<int64_t>(kRecIdLimit, live + need);
            rc = grow_recs(h, want);
            if (rc) return rc;
        }
    }
    out->rfreel = h->rfreel;
    out->rbase = h->rcursor;
    h->rcursor += need;
    return FS2_OK;
}

// An arena of at least `bytes` (grown by half again, the stream drained first:
// earlier transfers may still use the old one).  Sized at creation for the first
// resamples, so a timed scan normally never allocates.
static int ensure_arena(fs2_handle *h, char *&buf, size_t &cap, size_t bytes) {
    if (cap >= bytes) return FS2_OK;
    if (h->tp) scan_alloc(h, "scan_alloc arena (MiB)", bytes);   // (creation sizes it without a transport)
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    hipFree(buf);
    buf = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 2, 1 << 20);
    HIP_TRY(h, hipMalloc(&buf, want));
    cap = want;
    return FS2_OK;
}
static size_t arena_align(size_t b) { return (b + 255) & ~size_t(255); }

// Wait for a post (k_post / k_publish) whose flag reaches seq: spin for up to
// 50 ms, then fall back to a stream sync, which also reports a fault.
static int wait_seq(fs2_handle *h, const unsigned long long *flag, unsigned long long seq, const char *what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return FS2_OK;
        if ((it & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
        __builtin_ia32_pause();
    }
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) return set_err(&h->err, FS2_ERR_HIP, "%s were not posted", what);
    return FS2_OK;
}

// Sharded ranks, mid-scan: the statistics so far (the resample decision, the
// largest map on any rank) and, with xmat, the all-gathered transfer sizes, read
// through the post block.
static int post_and_wait(fs2_handle *h, bool sizes) {
    CommTimer ct(h);
    const int G = h->cfg.world_size;
    const unsigned long long seq = ++h->post_seq;
    HIP_TRY(h, launch_post(h->stats_dev, sizes ? h->xmat : nullptr, sizes ? kXrowWords * G * G : 0, h->post, h->post_flag_dev,
                           seq, h->stream));
    trace(h, "post wait", sizes ? 1 : 0);
    const int rc = wait_seq(h, h->post_flag, seq, "mid-scan statistics");
    trace(h, "posted", rc);
    if (rc) return rc;
    // k_post runs after the collectives queued before it, so a stream-ordered
    // transport's status is final here: a failed exchange leaves stale staging
    // bytes in the post, which must not size the resample
    return h->tp ? h->tp->status(&h->err) : FS2_OK;
}
static const DevStats &posted_stats(const fs2_handle *h) { return *reinterpret_cast<const DevStats *>(h->post_host); }
static const int64_t *posted_xmat(const fs2_handle *h) {
    return reinterpret_cast<const int64_t *>(h->post_host + sizeof(DevStats));
}

// The page-dedup table (XferTable) for `cap` slots and `nrows` row entries.
static int reserve_xfer_table(fs2_handle *h, int64_t cap, int64_t nrows, bool in_scan) {
    hipStream_t s = h->stream;
    if (in_scan && (h->xt_cap < cap || h->xt_ecap < nrows)) scan_alloc(h, "scan_alloc dedup table (M rows)", (size_t)nrows);
    if (h->xt_cap < cap) {
        HIP_TRY(h, hipStreamSynchronize(s));
        hipFree(h->xt_key); hipFree(h->xt_ref); hipFree(h->xt_uidx); hipFree(h->xt_cmask); hipFree(h->xt_cbase);
        h->xt_key = nullptr;
        h->xt_ref = h->xt_uidx = h->xt_cmask = h->xt_cbase = nullptr;
        h->xt_cap = 0;
        HIP_TRY(h, hipMalloc((void **)&h->xt_key, (size_t)cap * 8));
        // zeroed once here: page_refs' k_localize and the gather key it by epoch
        // (epoch 0 is never used) and never clear it, so a table allocated over
        // freed memory must not hold keys that look live
        HIP_TRY(h, hipMemsetAsync(h->xt_key, 0, (size_t)cap * 8, s));
        HIP_TRY(h, hipMalloc((void **)&h->xt_ref, (size_t)cap * 4));
        HIP_TRY(h, hipMalloc((void **)&h->xt_uidx, (size_t)cap * 4));
        HIP_TRY(h, hipMalloc((void **)&h->xt_cmask, (size_t)cap * 4));
        HIP_TRY(h, hipMalloc((void **)&h->xt_cbase, (size_t)cap * 4));
        h->xt_cap = cap;
    }
    if (h->xt_ecap < nrows) {
        HIP_TRY(h, hipStreamSynchronize(s));
        hipFree(h->xt_eslot); hipFree(h->xt_ulist);
        h->xt_eslot = h->xt_ulist = nullptr;
        h->xt_ecap = 0;
        const int64_t want = nrows + nrows / 4;
        HIP_TRY(h, hipMalloc((void **)&h->xt_eslot, (size_t)want * 4));
        HIP_TRY(h, hipMalloc((void **)&h->xt_ulist, (size_t)want * 4));
        h->xt_ecap = want;
    }
    return FS2_OK;
}

// The shard each rank keeps after a resample ("output shards follow
// their sources").  Systematic resampling keeps the global order, so the
// outputs of shard q are the children of one run of sources; with Q6/Q8's
// drift that run lies below q, on other ranks, and with shard r pinned to rank
// r nearly every rank would receive its whole shard.  Shards are the same size,
// so any one-to-one assignment of shards to ranks balances the work: take the
// one that keeps the most page-table rows local (the sum over ranks of the rows
// rank r's sources give shard keep_of[r]; ties keep the current shard, then
// the lower one).  An exact maximum by a DP over subsets of shards (2^G states,
// G <= 16), computed alike on every rank from the all-gathered counts.
template <typename At>
static void keep_shards(const fs2_handle *h, int G, At at, int keep_of[]) {
    int shard_of[kMaxRanks];
    for (int q = 0; q < G; ++q) shard_of[h->rank_of[q]] = q;
    if (!h->follow) {
        for (int r = 0; r < G; ++r) keep_of[r] = shard_of[r];
        return;
    }
    auto val = [&](int r, int q) { return 2 * at(r, q, 1) + (q == shard_of[r] ? 1 : 0); };
    const uint32_t full = (1u << G) - 1u;
    std::vector<int64_t> dp((size_t)full + 1, -1);
    std::vector<int8_t> pick((size_t)full + 1, -1);
    dp[0] = 0;
    for (uint32_t m = 0; m < full; ++m) {
        if (dp[m] < 0) continue;
        const int r = __builtin_popcount(m);      // ranks 0..r-1 are assigned
        for (int q = 0; q < G; ++q) {
            if (m & (1u << q)) continue;
            const uint32_t m2 = m | (1u << q);
            const int64_t v = dp[m] + val(r, q);
            if (v > dp[m2]) {
                dp[m2] = v;
                pick[m2] = (int8_t)q;
            }
        }
    }
    for (uint32_t m = full; m; m &= ~(1u << pick[m])) keep_of[__builtin_popcount(m) - 1] = pick[m];
}

// One resample's exchange, timed on the device when profiling (fs2_profile
// exchange_ms, recv_bytes: what must arrive before the next update pass).
static int timed_exchange(fs2_handle *h, const std::vector<fs2comm::Xfer> &sends,
                          const std::vector<fs2comm::Xfer> &recvs, hipStream_t s) {
    std::pair<hipEvent_t, hipEvent_t> *ev = nullptr;
    if (h->profiling) {
        if (h->xev_used == h->xev.size() && h->xev.size() < 256) {
            std::pair<hipEvent_t, hipEvent_t> e{nullptr, nullptr};
            if (hipEventCreate(&e.first) == hipSuccess && hipEventCreate(&e.second) == hipSuccess) h->xev.push_back(e);
            else (void)hipGetLastError();
        }
        if (h->xev_used < h->xev.size()) ev = &h->xev[h->xev_used++];
        for (const auto &x : recvs) h->prof.recv_bytes += x.bytes;
    }
    if (ev) HIP_TRY(h, hipEventRecord(ev->first, s));
    int rc;
    {
        CommTimer ct(h);
        rc = h->tp->exchange(sends, recvs, s, &h->err);
    }
    if (ev) HIP_TRY(h, hipEventRecord(ev->second, s));
    return rc;
}

// page_refs mode, after the sizes: each particle sent is its header and its rows
// as tagged descriptors (no page dedup, no page content, no second size round).
static int exchange_refs(fs2_handle *h, ResampleParams &rs, const std::vector<int64_t> &mat, int keep,
                         const int owner[], std::chrono::steady_clock::time_point t_start) {
    const int G = h->cfg.world_size, R = h->cfg.rank;
    hipStream_t s = h->stream;
    auto at = [&](int from, int to, int f) { return mat[(size_t)from * kXrowWords * G + kXrowWords * to + f]; };
    static const bool log_xfer = std::getenv("FS2_XFER_LOG") != nullptr;
    size_t soff[kMaxRanks + 1] = {}, roff[kMaxRanks + 1] = {};
    for (int p = 0; p < G; ++p) {
        const bool so = p != keep && at(R, p, 0) > 0, ro = p != R && at(p, keep, 0) > 0;
        soff[p + 1] = soff[p] + (so ? arena_align((size_t)xfer_ref_bytes(at(R, p, 0), at(R, p, 1))) : 0);
        roff[p + 1] = roff[p] + (ro ? arena_align((size_t)xfer_ref_bytes(at(p, keep, 0), at(p, keep, 1))) : 0);
    }
    int rc = ensure_arena(h, h->sarena, h->scap, soff[G]);
    if (!rc) rc = ensure_arena(h, h->rarena, h->rcap, roff[G]);
    if (rc) return rc;
    std::vector<fs2comm::Xfer> sends, recvs;
    int64_t nsend = 0;
    for (int p = 0; p < G; ++p) {
        rs.sbuf[p] = nullptr;
        const int64_t K = at(R, p, 0), S = at(R, p, 1);
        if (log_xfer)
            std::fprintf(stderr, "fs2 xfer (refs) scan %lld rank %d -> shard %d (rank %d)%s: %lld particles, %lld rows, %lld B\n",
                         (long long)h->scan, R, p, owner[p], p == keep ? " kept" : "", (long long)K, (long long)S,
                         (long long)(p == keep ? 0 : xfer_ref_bytes(K, S)));
        if (p == keep || K == 0) continue;
        rs.sbuf[p] = h->sarena + soff[p];
        sends.push_back({owner[p], rs.sbuf[p], (size_t)xfer_ref_bytes(K, S)});
        nsend += K;
    }
    if (nsend > INT32_MAX) return set_err(&h->err, FS2_ERR_CAPACITY, "%lld particles to send", (long long)nsend);
    HIP_TRY(h, launch_pack_refs(rs, s));
    rs.npeers = 0;
    int32_t kbase = 0;
    for (int q = 0; q < G; ++q) {
        if (q == R) continue;
        const int64_t K = at(q, keep, 0), S = at(q, keep, 1);
        if (!K) continue;
        char *rb = h->rarena + roff[q];
        recvs.push_back({q, rb, (size_t)xfer_ref_bytes(K, S)});
        RecvPeer &pp = rs.peers[rs.npeers++];
        pp = RecvPeer{};
        pp.pre = reinterpret_cast<const RefPreamble *>(rb);
        pp.hdr = reinterpret_cast<const PackHeader *>(rb + 64);
        pp.refs = reinterpret_cast<const XDesc *>(rb + 64 + 64 * K);
        pp.K = (int32_t)K;
        pp.kbase = kbase;
        kbase += (int32_t)K;
    }
    rc = timed_exchange(h, sends, recvs, s);
    if (rc) return rc;
    h->n_recv = kbase;
    h->u_recv = 0;
    h->refs_live = true;
    if (h->profiling) {
        uint64_t np = 0, nr = 0, nb = 0;
        for (int p = 0; p < G; ++p) {
            if (p == keep) continue;
            np += at(R, p, 0);
            nr += at(R, p, 1);
            nb += at(R, p, 0) ? xfer_ref_bytes(at(R, p, 0), at(R, p, 1)) : 0;
        }
        h->prof.migrations += np ? 1 : 0;
        h->prof.sent_particles += np;
        h->prof.sent_rows += nr;
        h->prof.sent_bytes += nb;
        h->prof.migrate_ms +=
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    }
    rs.ao = shard_begin(h->n_global, G, keep);
    if (h->follow) {
        ResampleParams r2 = rs;
        r2.ranges_mode = 2;
        HIP_TRY(h, launch_resample_ranges(r2, s));
    }
    if (keep != h->shard) h->shard_moves += 1;
    h->shard = keep;
    h->first = rs.ao;
    for (int q = 0; q < G; ++q) h->rank_of[q] = (int8_t)owner[q];
    return FS2_OK;
}

// Sharded resample: plan what goes to every other rank on the device (one run of
// local particles per destination, fs2_plan.hpp), all-gather the sizes and learn
// them with a post; find the distinct pages of every destination's rows
// (k_dedup_*), all-gather and learn their counts; pack all destinations in one
// pass and move them with one grouped exchange; then describe what arrived to the
// apply kernels.
static int exchange_particles(fs2_handle *h, ResampleParams &rs) {
    const int G = h->cfg.world_size, R = h->cfg.rank;
    const auto t_start = std::chrono::steady_clock::now();
    hipStream_t s = h->stream;
    rs.world = G;
    rs.rank = R;
    std::memcpy(rs.init_cov, h->cfg.init_landmark_cov, sizeof rs.init_cov);
    rs.plan = h->plan;
    rs.xrow = h->xrow;
    rs.sent_mask = h->sent_mask;
    HIP_TRY(h, launch_pack_count(rs, s));
    int rc;
    auto gather_sizes = [&]() -> int {
        {
            CommTimer ct(h);
            const int r = h->tp->allgather(h->xrow, h->xmat, sizeof(int64_t) * kXrowWords * G, s, &h->err);
            if (r) return r;
        }
        return post_and_wait(h, true);
    };
    rc = gather_sizes();
    if (rc) return rc;
    std::vector<int64_t> mat(posted_xmat(h), posted_xmat(h) + kXrowWords * G * G);
    // at(rank, shard, field): what rank `from` would send to the outputs of shard `to`
    auto at = [&](int from, int to, int f) { return mat[(size_t)from * kXrowWords * G + kXrowWords * to + f]; };
    // Which shard each rank keeps (its outputs are filled locally, not sent): every
    // rank computes the same assignment from the same counts (keep_shards)
    int keep_of[kMaxRanks], owner[kMaxRanks];
    keep_shards(h, G, at, keep_of);
    for (int r = 0; r < G; ++r) owner[keep_of[r]] = r;
    const int keep = keep_of[R];
    rs.keep = keep;
    // distinct pages of the rows sent (every rank takes part in the all-gather)
    XferTable &T = rs.xt;
    T = XferTable{};
    T.i_lo = h->n;
    T.i_hi = 0;
    for (int p = 0; p < G; ++p) {
        T.ebase[p + 1] = T.ebase[p] + (p == keep ? 0 : at(R, p, 1));
        if (p != keep && at(R, p, 0) > 0) {
            T.i_lo = std::min(T.i_lo, at(R, p, 4));
            T.i_hi = std::max(T.i_hi, at(R, p, 5));
        }
    }
    const int64_t nrows = T.ebase[G];
    if (h->refs) return exchange_refs(h, rs, mat, keep, owner, t_start);
    if (nrows > 0) {
        int lg = 10;
        while ((int64_t(1) << lg) < 2 * nrows) ++lg;
        if (lg > 31) return set_err(&h->err, FS2_ERR_CAPACITY, "%lld page-table rows to send", (long long)nrows);
        const int64_t cap = int64_t(1) << lg;
        rc = reserve_xfer_table(h, cap, nrows, true);
        if (rc) return rc;
        T.key = h->xt_key;
        T.ref = h->xt_ref;
        T.uidx = h->xt_uidx;
        T.cmask = h->xt_cmask;
        T.cbase = h->xt_cbase;
        T.eslot = h->xt_eslot;
        T.ulist = h->xt_ulist;
        T.cap = cap;
        T.log2cap = lg;
        HIP_TRY(h, hipMemsetAsync(T.key, 0, (size_t)cap * 8, s));
        HIP_TRY(h, hipMemsetAsync(T.ref, 0, (size_t)cap * 4, s));
        HIP_TRY(h, launch_pack_dedup(rs, s));
    }
    rc = gather_sizes();
    if (rc) return rc;
    mat.assign(posted_xmat(h), posted_xmat(h) + kXrowWords * G * G);
    static const bool log_xfer = std::getenv("FS2_XFER_LOG") != nullptr;
    int64_t nsend = 0;
    std::vector<fs2comm::Xfer> sends, recvs;
    // every destination's transfer at its offset in the send arena, every source's
    // in the receive arena
    size_t soff[kMaxRanks + 1] = {}, roff[kMaxRanks + 1] = {};
    // soff by destination shard, roff by source rank (sending to shard keep)
    for (int p = 0; p < G; ++p) {
        const bool so = p != keep && at(R, p, 0) > 0, ro = p != R && at(p, keep, 0) > 0;
        soff[p + 1] = soff[p] + (so ? arena_align((size_t)xfer_bytes(at(R, p, 0), at(R, p, 1), at(R, p, 2), at(R, p, 3))) : 0);
        roff[p + 1] = roff[p] + (ro ? arena_align((size_t)xfer_bytes(at(p, keep, 0), at(p, keep, 1), at(p, keep, 2),
                                                                      at(p, keep, 3))) : 0);
    }
    rc = ensure_arena(h, h->sarena, h->scap, soff[G]);
    if (!rc) rc = ensure_arena(h, h->rarena, h->rcap, roff[G]);
    if (rc) return rc;
    for (int p = 0; p < G; ++p) {
        rs.sbuf[p] = nullptr;
        T.ubase[p + 1] = T.ubase[p] + (p == keep ? 0 : at(R, p, 2));
        const int64_t K = at(R, p, 0), S = at(R, p, 1), U = at(R, p, 2), C = at(R, p, 3);
        if (log_xfer)
            std::fprintf(stderr,
                         "fs2 xfer scan %lld rank %d (shard %d -> %d) -> shard %d (rank %d)%s: %lld particles, "
                         "%lld rows, %lld pages, %lld covariances, %lld B\n",
                         (long long)h->scan, R, h->shard, keep, p, owner[p], p == keep ? " kept" : "", (long long)K,
                         (long long)S, (long long)U, (long long)C, (long long)(p == keep ? 0 : xfer_bytes(K, S, U, C)));
        if (p == keep || K == 0) continue;
        const size_t bytes = (size_t)xfer_bytes(K, S, U, C);
        rs.sbuf[p] = h->sarena + soff[p];
        sends.push_back({owner[p], rs.sbuf[p], bytes});
        nsend += K;
    }
    if (nsend > INT32_MAX) return set_err(&h->err, FS2_ERR_CAPACITY, "%lld particles to send", (long long)nsend);
    HIP_TRY(h, launch_pack_write(rs, s));
    rs.npeers = 0;
    int32_t kbase = 0;
    int64_t ubase = 0;
    for (int q = 0; q < G; ++q) {
        if (q == R) continue;
        const int64_t K = at(q, keep, 0), S = at(q, keep, 1), U = at(q, keep, 2), C = at(q, keep, 3);
        if (!K) continue;
        const size_t bytes = (size_t)xfer_bytes(K, S, U, C);
        char *rb = h->rarena + roff[q];
        recvs.push_back({q, rb, bytes});
        RecvPeer &pp = rs.peers[rs.npeers++];
        pp.hdr = reinterpret_cast<const PackHeader *>(rb);
        pp.idx = reinterpret_cast<const uint32_t *>(rb + xfer_idx_off(K));
        pp.pages = reinterpret_cast<const XferPage *>(rb + xfer_page_off(K, S));
        pp.covs = reinterpret_cast<const double2 *>(rb + xfer_cov_off(K, S, U));
        pp.K = (int32_t)K;
        pp.kbase = kbase;
        pp.U = U;
        pp.ubase = ubase;
        kbase += (int32_t)K;
        ubase += U;
    }
    rc = timed_exchange(h, sends, recvs, s);
    if (rc) return rc;
    h->n_recv = kbase;
    h->u_recv = ubase;
    if (h->profiling) {
        uint64_t np = 0, nr = 0, nu = 0, nb = 0;
        for (int p = 0; p < G; ++p) {
            if (p == keep) continue;
            np += at(R, p, 0);
            nr += at(R, p, 1);
            nu += at(R, p, 2);
            nb += at(R, p, 0) ? xfer_bytes(at(R, p, 0), at(R, p, 1), at(R, p, 2), at(R, p, 3)) : 0;
        }
        h->prof.migrations += np ? 1 : 0;
        h->prof.sent_particles += np;
        h->prof.sent_rows += nr;
        h->prof.sent_pages += nu;
        h->prof.sent_bytes += nb;
        h->prof.migrate_ms +=
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    }
    // this rank now holds shard keep: its local outputs (the local sources'
    // outputs inside that shard) are filled relative to the shard's start
    rs.ao = shard_begin(h->n_global, G, keep);
    if (h->follow) {
        ResampleParams r2 = rs;
        r2.ranges_mode = 2;
        HIP_TRY(h, launch_resample_ranges(r2, s));
    }
    if (keep != h->shard) h->shard_moves += 1;
    h->shard = keep;
    h->first = rs.ao;
    for (int q = 0; q < G; ++q) h->rank_of[q] = (int8_t)owner[q];
    return FS2_OK;
}

// Layout of an imported map: slots in an order whose runs of 8
// (one page each) are spatially compact, so that page boxes are small and the
// candidate stream opens few pages.  Recursive bisection: split the set along
// its longer extent at a multiple of 8 near the middle.  The slot index travels
// in each mirror, so the layout never changes a result; maps with non-finite
// coordinates keep slot order.
static bool spatial_order(const double *lm, int L, std::vector<int32_t> &perm) {
    perm.resize(L);
    for (int j = 0; j < L; ++j) {
        perm[j] = j;
        if (!std::isfinite(lm[6 * j]) || !std::isfinite(lm[6 * j + 1])) return false;
    }
    struct Rec {
        static void go(const double *lm, int32_t *a, int n) {
            if (n <= kPageSlots) return;
            double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
            for (int k = 0; k < n; ++k) {
                x0 = std::min(x0, lm[6 * a[k]]);
                x1 = std::max(x1, lm[6 * a[k]]);
                y0 = std::min(y0, lm[6 * a[k] + 1]);
                y1 = std::max(y1, lm[6 * a[k] + 1]);
            }
            const int ax = (x1 - x0 >= y1 - y0) ? 0 : 1;
            std::stable_sort(a, a + n, [&](int32_t u, int32_t v) { return lm[6 * u + ax] < lm[6 * v + ax]; });
            int h = ((n / 2 + kPageSlots - 1) / kPageSlots) * kPageSlots;
            if (h >= n) h = n - kPageSlots;
            go(lm, a, h);
            go(lm, a + h, n - h);
        }
    };
    Rec::go(lm, perm.data(), L);
    return true;
}

extern "C" {

int32_t fs2_abi_version(void) { return FS2_ABI_VERSION; }

#ifndef FS2_BUILD_ID
#define FS2_BUILD_ID "unknown"
#endif
const char *fs2_build_id(void) { return FS2_BUILD_ID; }

void fs2_config_default(fs2_config *c) {
    if (!c) return;
    std::memset(c, 0, sizeof *c);
    c->num_particles = 20;                 // config.py:7
    c->translation_noise = 0.0055;         // config.py:11
    c->rotation_noise = 0.001;             // config.py:12
    c->measurement_noise[0] = 0.001;       // config.py:15
    c->measurement_noise[3] = 0.001;
    c->max_landmark_distance = 8.0;        // config.py:18
    c->init_landmark_cov[0] = 0.1;         // landmark.py:13
    c->init_landmark_cov[3] = 0.1;
    c->weight_floor = 1e-5;                // fast_slam_2.py:168,173
    c->landmark_capacity = 64;
    c->max_landmark_capacity = 4096;
    c->device = 0;
    c->reduce_mode = FS2_REDUCE_AUTO;
    c->seed = 0x5EEDF5A2ull;
    c->record_assoc = 0;
    c->gate_filter = 1;
    c->rank = 0;
    c->world_size = 1;
}

const char *fs2_last_error(const fs2_handle *h) {
    if (h && !h->err.empty()) return h->err.c_str();
    return g_last_error.c_str();
}

static void free_handle(fs2_handle *h) {
    if (!h) return;
    // the handle's device is current while it is torn down (the device-wide
    // synchronisations below must drain *its* device; ranks of one process may sit
    // on several GPUs), and the caller's device is restored at the end
    int prev_dev = -1;
    if (hipGetDevice(&prev_dev) != hipSuccess) prev_dev = -1;
    if (prev_dev != h->cfg.device) (void)hipSetDevice(h->cfg.device);
    if (h->stream) hipStreamSynchronize(h->stream);
    if (h->mt.dstream) hipStreamSynchronize(h->mt.dstream);   // (a deferred draw)
    // In-place pools (VMM chunks): nothing of this process may still be in flight
    // when they are unmapped and released, or the runtime defers the release and the
    // next handle's first growth (hipMemCreate) waits for it -- 4 s in the round-4
    // driver bench (profiles/r04_g8_refs_growth_probe.txt; a device synchronize
    // between the sets of handles brought it back to milliseconds).
    const bool vmm = h->pool_vm.base || h->rpool_vm.base || h->freel_vm.base || h->mark_vm.base ||
                     h->rfreel_vm.base || h->rmark_vm.base;
    if (vmm) hipDeviceSynchronize();
    if (h->refs_shared && h->tp && !h->tp->in_process()) {
        // page_refs: no rank frees its pools while another may still read them (an
        // export of maps naming remote pages): every rank arrives, unmaps the others'
        // pools, arrives again (a failed transport skips the rendezvous).  Ranks that
        // are threads of one process are closed one by one: their caller closes them
        // after the last export
        std::string e;
        if (h->tp->allgather(h->ep_dev, h->epochs_dev, 1, h->stream, &e) == FS2_OK) hipStreamSynchronize(h->stream);
        h->tp->unshare();
        if (h->tp->allgather(h->ep_dev, h->epochs_dev, 1, h->stream, &e) == FS2_OK) hipStreamSynchronize(h->stream);
    }
    for (int s = 0; s < 2; ++s) {
        hipFree(h->x[s]); hipFree(h->y[s]); hipFree(h->yaw[s]); hipFree(h->w[s]); hipFree(h->cnt[s]);
        hipFree(h->pt[s]);
        hipFree(h->bbox[s]);
    }
    hipFree(h->rdesc); hipFree(h->udesc);
    hipFree(h->xt_key); hipFree(h->xt_ref); hipFree(h->xt_uidx); hipFree(h->xt_cmask); hipFree(h->xt_cbase);
    hipFree(h->xt_eslot); hipFree(h->xt_ulist);
    hipFree(h->sent_mask);
    if (h->pool_vm.base) gm_free(h->pool_vm);
    else hipFree(h->pool);
    if (h->rpool_vm.base) gm_free(h->rpool_vm);
    else hipFree(h->rpool);
    if (h->freel_vm.base) gm_free(h->freel_vm); else hipFree(h->freel);
    if (h->mark_vm.base) gm_free(h->mark_vm); else hipFree(h->mark);
    if (h->rfreel_vm.base) gm_free(h->rfreel_vm); else hipFree(h->rfreel);
    if (h->rmark_vm.base) gm_free(h->rmark_vm); else hipFree(h->rmark);
    if (vmm) hipDeviceSynchronize();       // (the releases complete here, not at the next growth)
    hipFree(h->bcnt); hipFree(h->nfree_dev);
    hipFree(h->rbcnt); hipFree(h->rnfree_dev);
    hipFree(h->slb); hipFree(h->slb_pass); hipFree(h->ext_dev);
    hipFree(h->rank_d); hipFree(h->rank_e); hipFree(h->iblk);
    hipFree(h->mlo); hipFree(h->mhi); hipFree(h->out_src); hipFree(h->runs); hipFree(h->runs_n);
    hipFree(h->rec); hipFree(h->recs); hipFree(h->totals); hipFree(h->xrow); hipFree(h->xmat);
    hipFree(h->sarena);
    hipFree(h->rarena);
    hipFree(h->cand); hipFree(h->ncand);
    hipFree(h->uinfo); hipFree(h->uol); hipFree(h->seql); hipFree(h->udelta); hipFree(h->ugl);
    hipFree(h->bD); hipFree(h->bC); hipFree(h->bM); hipFree(h->bpd); hipFree(h->bpc);
    hipFree(h->uel); hipFree(h->bE); hipFree(h->bpe);
    hipFree(h->sout); hipFree(h->np_leaf); hipFree(h->part_w); hipFree(h->np_part); hipFree(h->np_tail);
    hipFree(h->urec); hipFree(h->sentry);
    hipFree(h->dch_send); hipFree(h->dch_recv); hipFree(h->recx); hipFree(h->recxs); hipFree(h->est_base);
    hipFree(h->uop); hipFree(h->np_tail_g);
    hipFree(h->peers_dev); hipFree(h->ep_dev); hipFree(h->epochs_dev);
    hipFree(h->part_pose);
    hipFree(h->gen_dev); hipFree(h->sets_dev); hipFree(h->go_dev);
    hipFree(h->wpart); hipFree(h->cpart); hipFree(h->part_sq); hipFree(h->part_best_w); hipFree(h->part_best_i); hipFree(h->part_slots);
    hipFree(h->part_maxcnt); hipFree(h->cbuf); hipFree(h->bsum);
    hipFree(h->stats_dev); hipFree(h->noise_dev); hipFree(h->u0_dev); hipFree(h->assoc_dev);
    if (h->post_host) hipHostFree(h->post_host);
    hipFree(h->plan);
    if (h->pub_stats) hipHostFree(h->pub_stats);
    if (h->noise_pin) hipHostFree(h->noise_pin);
    if (h->u0_pin) hipHostFree(h->u0_pin);
    if (h->mt.side) hipStreamSynchronize(h->mt.side);
    if (h->mt.dstream) {
        hipStreamSynchronize(h->mt.dstream);
        hipStreamDestroy(h->mt.dstream);
        hipEventDestroy(h->mt.ev_in);
        hipEventDestroy(h->mt.ev_noise);
    }
    hipFree(h->mt.raw[0]); hipFree(h->mt.raw[1]); hipFree(h->mt.boff);
    if (h->mt.ev_words) hipEventDestroy(h->mt.ev_words);
    if (h->mt.ev_pre) hipEventDestroy(h->mt.ev_pre);
    if (h->mt.side) hipStreamDestroy(h->mt.side); hipFree(h->mt.meta); hipFree(h->mt.amb); hipFree(h->mt.pidx);
    hipFree(h->mt.pval); hipFree(h->mt.tab); hipFree(h->mt.jpoly); hipFree(h->mt.jwin);
    if (h->mt.meta_pin) hipHostFree(h->mt.meta_pin);
    if (h->mt.amb_pin) hipHostFree(h->mt.amb_pin);
    if (h->mt.words_pin) hipHostFree(h->mt.words_pin);
    if (h->mt.pidx_pin) hipHostFree(h->mt.pidx_pin);
    if (h->mt.pval_pin) hipHostFree(h->mt.pval_pin);
    if (h->ev.ok)
        for (auto &set : h->ev.e)
            for (auto &e : set) hipEventDestroy(e);
    for (auto &e : h->xev) {
        hipEventDestroy(e.first);
        hipEventDestroy(e.second);
    }
    delete h->tp;
    if (h->stream) hipStreamDestroy(h->stream);
    const int dev = h->cfg.device;
    delete h;
    if (prev_dev >= 0 && prev_dev != dev) (void)hipSetDevice(prev_dev);
}

int fs2_create(const fs2_config *cfg, fs2_handle **out) {
    if (!cfg || !out) return set_err(nullptr, FS2_ERR_ARG, "fs2_create: null argument");
    *out = nullptr;
    if (cfg->num_particles <= 0)
        return set_err(nullptr, FS2_ERR_ARG, "num_particles must be positive");
    if (cfg->world_size < 1 || cfg->rank < 0 || cfg->rank >= cfg->world_size)
        return set_err(nullptr, FS2_ERR_ARG, "bad rank %d / world_size %d", cfg->rank, cfg->world_size);
    if (cfg->world_size > kMaxRanks)
        return set_err(nullptr, FS2_ERR_ARG, "world_size %d > %d", cfg->world_size, kMaxRanks);
    if (cfg->num_particles > (int64_t)INT32_MAX)
        return set_err(nullptr, FS2_ERR_ARG, "too many particles per rank");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return set_err(nullptr, FS2_ERR_HIP, "no HIP device available (libfs2 has no CPU path)");
    if (cfg->device < 0 || cfg->device >= ndev)
        return set_err(nullptr, FS2_ERR_ARG, "device %d out of range (%d devices)", cfg->device, ndev);

    fs2_handle *h = new fs2_handle();
    h->cfg = *cfg;
    h->n_global = cfg->num_particles;
    const int64_t G = cfg->world_size, r = cfg->rank;
    h->first = (h->n_global * r) / G;
    h->n = (h->n_global * (r + 1)) / G - h->first;
    h->shard = (int32_t)r;
    for (int q = 0; q < kMaxRanks; ++q) h->rank_of[q] = (int8_t)(q < G ? q : 0);
    // shards can change hands only when they are all the same size (buffers are
    // sized for n); FS2_SHARD_FOLLOW=0 pins shard r to rank r (A/B)
    {
        const char *e = std::getenv("FS2_SHARD_FOLLOW");
        h->follow = G > 1 && h->n_global % G == 0 && !(e && std::strcmp(e, "0") == 0);
    }
    h->max_cap = cfg->max_landmark_capacity > 0 ? std::min(cfg->max_landmark_capacity, kMaxSlots) : kMaxSlots;
    h->gate2 = gate_to_q(cfg->max_landmark_distance);
    auto fail = [&](int code) {
        std::string msg = h->err;
        free_handle(h);
        g_last_error = msg;
        return code;
    };
    if (hipSetDevice(cfg->device) != hipSuccess) return fail(set_err(&h->err, FS2_ERR_HIP, "hipSetDevice failed"));
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
        return fail(set_err(&h->err, FS2_ERR_HIP, "hipStreamCreate failed"));
    const int64_t n = std::max<int64_t>(h->n, 1);
    const int64_t nb = (n + kBlock - 1) / kBlock;
    const int64_t nsb = (n + 1023) / 1024;
    // FS2_GUARD=1 (tests): every buffer below is followed by kGuardBytes of a known
    // pattern that fs2_debug_check_guards verifies -- a kernel writing past the end
    // of one of them is found by name instead of by a fault (or by nothing)
    const bool guard = [] {
        const char *e = std::getenv("FS2_GUARD");
        return e && *e && std::strcmp(e, "0") != 0;
    }();
    auto alloc = [&](void **p, size_t bytes, const char *name) {
        const size_t b = bytes > 0 ? bytes : 16, tot = guard ? b + kGuardBytes : b;
        hipError_t e = hipMalloc(p, tot);
        if (e == hipErrorOutOfMemory && g_chunks.release() > 0) {   // closed handles' kept chunks
            (void)hipGetLastError();
            e = hipMalloc(p, tot);
        }
        if (e == hipSuccess && guard) {
            e = hipMemset(static_cast<char *>(*p) + b, kGuardByte, kGuardBytes);
            h->guards.push_back(fs2_handle::Guard{static_cast<char *>(*p) + b, name});
        }
        return e;
    };
#define FS2_ALLOC(ptr, bytes) alloc((void **)&(ptr), (size_t)(bytes), #ptr)
    bool ok = true;
    for (int s = 0; s < 2; ++s) {
        ok &= FS2_ALLOC(h->x[s], n * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->y[s], n * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->yaw[s], n * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->w[s], n * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->cnt[s], n * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->bbox[s], nb * kBBoxRows * 4) == hipSuccess;
    }
    ok &= FS2_ALLOC(h->nfree_dev, sizeof(int64_t)) == hipSuccess;
    ok &= FS2_ALLOC(h->rnfree_dev, sizeof(int64_t)) == hipSuccess;
    ok &= FS2_ALLOC(h->slb, sizeof(float)) == hipSuccess;
    ok &= FS2_ALLOC(h->slb_pass, sizeof(float)) == hipSuccess;
    ok &= FS2_ALLOC(h->ext_dev, sizeof(uint32_t)) == hipSuccess;
    ok &= FS2_ALLOC(h->mlo, n * 4) == hipSuccess;
    ok &= FS2_ALLOC(h->mhi, n * 4) == hipSuccess;
    ok &= FS2_ALLOC(h->out_src, n * 4) == hipSuccess;
    ok &= FS2_ALLOC(h->runs, sizeof(int4) * kMaxLongRuns) == hipSuccess;
    ok &= FS2_ALLOC(h->runs_n, 4) == hipSuccess && hipMemset(h->runs_n, 0, 4) == hipSuccess;
    ok &= FS2_ALLOC(h->cand, n * 8 * kMaxCand) == hipSuccess;
    ok &= FS2_ALLOC(h->ncand, n * 4) == hipSuccess;
    ok &= FS2_ALLOC(h->rec, sizeof(RankRecord)) == hipSuccess;
    ok &= FS2_ALLOC(h->recs, sizeof(RankRecord) * G) == hipSuccess;
    ok &= FS2_ALLOC(h->totals, sizeof(double) * G) == hipSuccess;
    ok &= FS2_ALLOC(h->xrow, sizeof(int64_t) * kXrowWords * G) == hipSuccess;
    ok &= FS2_ALLOC(h->xmat, sizeof(int64_t) * kXrowWords * G * G) == hipSuccess;
    ok &= FS2_ALLOC(h->rank_d, n * 4) == hipSuccess;
    ok &= FS2_ALLOC(h->rank_e, n * 4) == hipSuccess;
    ok &= FS2_ALLOC(h->iblk, (2 * nsb + 2) * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->wpart, nb * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->cpart, 2 * nb * 8 * kNumCounters) == hipSuccess;   // [2]: by scan parity
    ok &= FS2_ALLOC(h->gen_dev, 4) == hipSuccess;
    ok &= FS2_ALLOC(h->go_dev, 8) == hipSuccess;
    ok &= FS2_ALLOC(h->sets_dev, 2 * sizeof(BufSet)) == hipSuccess;
    ok &= FS2_ALLOC(h->part_sq, nb * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->part_best_w, nb * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->part_pose, nb * 24) == hipSuccess;
    ok &= FS2_ALLOC(h->part_best_i, nb * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->part_slots, nb * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->part_maxcnt, nb * 4) == hipSuccess;
    ok &= FS2_ALLOC(h->cbuf, n * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->bsum, nsb * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->stats_dev, sizeof(DevStats)) == hipSuccess;
    {
        const int64_t nu = (n + 63) / 64;
        ok &= FS2_ALLOC(h->uinfo, nu * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->uol, nu * 4) == hipSuccess;
        const int64_t ng = (nu + kChainGroup - 1) / kChainGroup;
        ok &= FS2_ALLOC(h->bD, ng * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->bC, ng * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->bM, ng * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->bpd, ng * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->bpc, ng * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->uel, nu * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->bE, ng * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->bpe, ng * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->seql, nu * 4) == hipSuccess;
        ok &= FS2_ALLOC(h->udelta, nu * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->ugl, nu * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->sout, nu * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->sentry, nu * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->urec, nu * sizeof(UnitRec)) == hipSuccess;
        ok &= FS2_ALLOC(h->np_leaf, (np_sumsq_chunks(n) * 64 + 64) * 8) == hipSuccess;
        ok &= FS2_ALLOC(h->part_w, nb * 8) == hipSuccess;
        // (one sum per numpy chunk in the tree modes, one per half chunk in the
        // chunked exact mode: k_normalize_chunks writes normalize_chunk_parts(n) --
        // sized by chunks alone, the N = 8e6 drift study's first scan wrote past it
        // and faulted; at N = 1e6 the overrun stayed inside the allocation's granule)
#ifdef FS2_AB_OLD_NP_PART            // (the round-5 size: validates FS2_GUARD against the real overrun)
        ok &= FS2_ALLOC(h->np_part, np_sumsq_chunks(n) * 8) == hipSuccess;
#else
        ok &= FS2_ALLOC(h->np_part,
                    std::max<int64_t>(np_sumsq_chunks(n), normalize_chunk_parts(n)) * 8) == hipSuccess;
#endif
    }
    ok &= FS2_ALLOC(h->noise_dev, n * 8) == hipSuccess;
    ok &= FS2_ALLOC(h->u0_dev, 8) == hipSuccess;
    {
        // post block: DevStats, xmat (kXrowWords G x G words), then the flag on its own line
        const size_t body = sizeof(DevStats) + sizeof(int64_t) * kXrowWords * kMaxRanks * kMaxRanks;
        const size_t off = ((body + 63) / 64) * 64;
        ok &= hipHostMalloc((void **)&h->post_host, off + 128, hipHostMallocCoherent | hipHostMallocMapped) ==
              hipSuccess;
        if (ok) {
            h->post_flag = reinterpret_cast<unsigned long long *>(h->post_host + off);
            *h->post_flag = 0;
            ok &= hipHostGetDevicePointer((void **)&h->post, h->post_host, 0) == hipSuccess;
            if (ok) h->post_flag_dev = reinterpret_cast<unsigned long long *>(h->post + off);
        }
    }
    ok &= FS2_ALLOC(h->plan, sizeof(PackPlan) * kMaxRanks) == hipSuccess;
    // one coherent block: the published stats, then the flag on its own 64-byte line
    ok &= hipHostMalloc((void **)&h->pub_stats, sizeof(DevStats) + 128, hipHostMallocCoherent | hipHostMallocMapped) ==
          hipSuccess;
    if (ok) {
        const size_t off = ((sizeof(DevStats) + 63) / 64) * 64;
        h->pub_flag = reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(h->pub_stats) + off);
        *h->pub_flag = 0;
        ok &= hipHostGetDevicePointer((void **)&h->pub_stats_dev, h->pub_stats, 0) == hipSuccess;
        if (ok)
            h->pub_flag_dev = reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(h->pub_stats_dev) + off);
    }
    ok &= hipHostMalloc((void **)&h->noise_pin, 2 * n * 8, 0) == hipSuccess;   // [2]: by scan parity
    ok &= hipHostMalloc((void **)&h->u0_pin, 2 * 8, 0) == hipSuccess;
    if (!ok) return fail(set_err(&h->err, FS2_ERR_OOM, "device allocation failed for %lld particles", (long long)n));
    if (hipMemsetAsync(h->cpart, 0, 2 * nb * 8 * kNumCounters, h->stream) != hipSuccess ||
        hipMemsetAsync(h->gen_dev, 0, 4, h->stream) != hipSuccess ||
        hipMemsetAsync(h->go_dev, 0, 8, h->stream) != hipSuccess ||
        hipMemsetD32Async((hipDeviceptr_t)h->slb, 0x7f7fffff, 1, h->stream) != hipSuccess)   // FLT_MAX: no mirror yet
        return fail(set_err(&h->err, FS2_ERR_HIP, "state initialisation failed"));
    // Particle.__init__: (0, 0, 0), weight 1/NUM_PARTICLES, empty map (particle.py:11-20)
    for (int s = 0; s < 2; ++s) {
        if (hipMemsetAsync(h->x[s], 0, n * 8, h->stream) != hipSuccess ||
            hipMemsetAsync(h->y[s], 0, n * 8, h->stream) != hipSuccess ||
            hipMemsetAsync(h->yaw[s], 0, n * 8, h->stream) != hipSuccess ||
            hipMemsetAsync(h->cnt[s], 0, n * 4, h->stream) != hipSuccess ||
            hipMemsetD32Async((hipDeviceptr_t)h->bbox[s], (int)kBoxEmpty, nb * kBBoxRows, h->stream) != hipSuccess ||
            launch_fill(h->w[s], 1.0 / (double)h->n_global, n, h->stream) != hipSuccess)
            return fail(set_err(&h->err, FS2_ERR_HIP, "state initialisation failed"));
    }
    {
        NpTailPlan plan;
        if (np_tail_plan(h->n, &plan)) {
            if (hipMalloc(&h->np_tail, sizeof plan) != hipSuccess ||
                hipMemcpy(h->np_tail, &plan, sizeof plan, hipMemcpyHostToDevice) != hipSuccess)
                return fail(set_err(&h->err, FS2_ERR_HIP, "state initialisation failed"));
        }
    }
    if (G > 1) {
        // exact reductions across shards: every shard holds at least one numpy chunk
        // (a chunk is then cut by at most one shard boundary) and at most kShardChunks
        // whole chunks, and the global partial chunk's plan fits an edge record
        NpTailPlan gp;
        const bool gpart = np_tail_plan(h->n_global, &gp);
        const int64_t min_shard = h->n_global / G, max_shard = (h->n_global + G - 1) / G;
        h->xsh_ok = min_shard >= kNpChunk && max_shard / kNpChunk + 1 <= kShardChunks && (!gpart || gp.nl <= 128);
        if (cfg->reduce_mode == FS2_REDUCE_EXACT && !h->xsh_ok)
            return fail(set_err(&h->err, FS2_ERR_ARG,
                                "exact reductions across %d shards need >= %d particles per shard (%lld)",
                                (int)G, kNpChunk, (long long)min_shard));
        if (h->xsh_ok) {
            const int64_t nu = (n + 63) / 64;      // chain units (kUnit)
            bool ok2 = hipMalloc(&h->dch_send, sizeof(ChainSummary)) == hipSuccess &&
                       hipMalloc(&h->dch_recv, sizeof(ChainSummary) * G) == hipSuccess &&
                       hipMalloc(&h->recx, sizeof(RankRecordX)) == hipSuccess &&
                       hipMalloc(&h->recxs, sizeof(RankRecordX) * G) == hipSuccess &&
                       hipMalloc(&h->est_base, sizeof(double)) == hipSuccess &&
                       hipMalloc(&h->uop, sizeof(int32_t) * (size_t)std::max<int64_t>(nu, 1)) == hipSuccess;
            if (ok2 && gpart)
                ok2 = hipMalloc(&h->np_tail_g, sizeof gp) == hipSuccess &&
                      hipMemcpy(h->np_tail_g, &gp, sizeof gp, hipMemcpyHostToDevice) == hipSuccess;
            if (ok2) ok2 = hipMemset(h->recx, 0, sizeof(RankRecordX)) == hipSuccess;
            if (!ok2) return fail(set_err(&h->err, FS2_ERR_OOM, "sharded reduction buffers"));
        }
    }
    int rc = grow_rows(h, std::max(cfg->landmark_capacity, 1));
    if (rc) return fail(rc);
    // pool: twice the initial maps plus room for a few scans of new pages;
    // records: the initial maps plus room for many scans of writes; a sharded
    // rank also room to receive half its shard's maps without sharing (the first
    // resamples, before the particles share ancestors), so that no resample
    // grows a pool (a large hipMalloc and copy: hundreds of ms)
    // (page_refs mode: the same room serves the pages localised from other ranks)
    const int64_t recv_pages = G > 1 ? n / 2 * h->rows : 0;
    const int64_t recv_recs = G > 1 ? n / 2 * h->rows * kPageSlots : 0;
    int64_t npages = cfg->page_pool > 0 ? cfg->page_pool : n * h->rows * 2 + 8 * n + recv_pages + 1024;
    // page_refs mode (fs2.h): 2..15 ranks, local page ids below 2^27 (the rank tag
    // above them); a default pool is clamped to the id space while it still holds
    // the initial maps 1.25 times over, else the mode stays off (auto) or fails (on)
    // on request only (page_refs = 1).  Measured in round 4: a
    // resample sends ~10x fewer bytes, but the update passes then localise remote
    // pages one particle-row at a time (siblings that share a remote page each copy
    // it), which moved more bytes and took longer per scan than sending each
    // distinct page once.  Between processes the pools are VMM chunks exported
    // as file descriptors (vm_share, Transport::share_vm): the runtime's
    // hipIpcOpenMemHandle did not return in a process that had exported an
    // allocation itself (profiles/r05_ipc_probe.txt).
    const bool refs_wanted = cfg->page_refs == 1;
    if (G > 1 && refs_wanted) {
        const int64_t lim = (int64_t)kRefIdMask - 1024;
        if (cfg->page_pool <= 0 && npages > lim && lim >= n * h->rows + n * h->rows / 4 + 8 * n) npages = lim;
        h->refs = G <= kRefMaxRanks && npages <= lim;
        h->vm_share = h->refs && cfg->comm_mode != FS2_COMM_LOCAL;
        // pools shared with the peers never grow: room for a few more scans of
        // reservations between the collective collections
        if (h->refs && cfg->page_pool <= 0) npages = std::min(lim, npages + 24 * n);
        if (cfg->page_refs == 1 && !h->refs)
            return fail(set_err(&h->err, FS2_ERR_ARG, "page_refs: needs 2..%d ranks and a page pool below %lld pages",
                                kRefMaxRanks, (long long)lim));
    }
    rc = grow_pool(h, npages);
    if (rc) return fail(rc);
    rc = grow_recs(h, cfg->record_pool > 0 ? cfg->record_pool
                                            : n * h->cap + n * h->cap / 4 + 64 * n + recv_recs + 1024 +
                                                  (h->refs ? 24 * n : 0));
    if (rc) return fail(rc);
    if (G > 1) {
        // the sharded resample's buffers, made here rather than in a timed scan: the
        // dedup table, the send and receive arenas for half the shard with nothing
        // shared (the first resamples move up to ~40 % of a rank's particles, to up
        // to three ranks), and the received particles' rows and pages
        const int64_t K = n / 2 + 1, S = K * h->rows;
        rc = xfer_bufs(h);
        const size_t bytes = (size_t)xfer_bytes(K, S, S, 0) + 256 * kMaxRanks;
        if (!rc) rc = ensure_arena(h, h->sarena, h->scap, bytes);
        if (!rc) rc = ensure_arena(h, h->rarena, h->rcap, bytes);
        if (rc) return fail(rc == FS2_ERR_OOM ? set_err(&h->err, rc, "sharded transfer buffers") : rc);
    }
    if (G > 1 || cfg->sharded_path) {
        rc = (cfg->comm_mode == FS2_COMM_LOCAL) ? fs2comm::create_local(cfg->comm_id, (int)G, (int)r, &h->tp, &h->err)
             : (cfg->comm_mode == FS2_COMM_SHM) ? fs2comm::create_shm(cfg->comm_id, (int)G, (int)r, &h->tp, &h->err)
                                                 : fs2comm::create_rccl(cfg->comm_id, (int)G, (int)r, &h->tp, &h->err);
        if (rc) return fail(rc);
    }
    if (h->refs &&
        (hipMalloc(&h->peers_dev, sizeof(PeerMaps)) != hipSuccess || hipMalloc(&h->ep_dev, 64) != hipSuccess ||
         hipMalloc(&h->epochs_dev, 2 * kMaxRanks) != hipSuccess))
        return fail(set_err(&h->err, FS2_ERR_OOM, "page_refs tables"));
    if (hipStreamSynchronize(h->stream) != hipSuccess)
        return fail(set_err(&h->err, FS2_ERR_HIP, "initialisation sync failed"));
    *out = h;
    return FS2_OK;
}

void fs2_destroy(fs2_handle *h) { free_handle(h); }

int fs2_shard_info(const fs2_handle *h, int64_t *n_local, int64_t *first_global, int32_t *capacity) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    if (n_local) *n_local = h->n;
    if (first_global) *first_global = h->first;
    if (capacity) *capacity = h->cap;
    return FS2_OK;
}

int fs2_synchronize(fs2_handle *h) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    return FS2_OK;
}

int fs2_set_profiling(fs2_handle *h, int32_t enable) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    if (h->pending.on) return set_err(&h->err, FS2_ERR_STATE, "a submitted scan is pending (fs2_iterate_wait first)");
    if (enable && !h->ev.ok) {
        for (auto &set : h->ev.e)
            for (auto &e : set) HIP_TRY(h, hipEventCreate(&e));
        h->ev.ok = true;
    }
    h->ev.used = 0;
    h->xev_used = 0;
    h->profiling = enable > 0;
    h->prof_period = enable > 0 ? enable : 1;
    h->prof_tick = 0;
    h->prof = fs2_profile{};
    return FS2_OK;
}

static int fold_profile(fs2_handle *h);

int fs2_get_profile(const fs2_handle *hc, fs2_profile *out) {
    if (!hc || !out) return set_err(nullptr, FS2_ERR_ARG, "null argument");
    fs2_handle *h = const_cast<fs2_handle *>(hc);   // the last scan's events are folded in
    if (h->pending.on) return set_err(&h->err, FS2_ERR_STATE, "a submitted scan is pending (fs2_iterate_wait first)");
    const int rc = fold_profile(h);
    if (rc) return rc;
    for (size_t k = 0; k < h->xev_used; ++k) {
        float ms = 0.0f;
        HIP_TRY(h, hipEventSynchronize(h->xev[k].second));
        HIP_TRY(h, hipEventElapsedTime(&ms, h->xev[k].first, h->xev[k].second));
        h->prof.exchange_ms += ms;
    }
    h->xev_used = 0;
    *out = h->prof;
    out->page_refs = h->refs_off ? -1 : (h->refs ? 1 : 0);
    return FS2_OK;
}

static int fold_one(fs2_handle *h, int set);

// Adds every profiled scan not yet folded (ProfEvents) to h->prof.
static int fold_profile(fs2_handle *h) {
    const int used = h->ev.used;
    h->ev.used = 0;
    for (int k = 0; k < used; ++k) {
        const int rc = fold_one(h, k);
        if (rc) return rc;
    }
    return FS2_OK;
}

static int fold_one(fs2_handle *h, int set) {
    const ProfScan &p = h->ev.scan[set];
    hipEvent_t *E = h->ev.e[set];
    HIP_TRY(h, hipEventSynchronize(E[3]));
    const DevStats &st = p.st;
    float a = 0, f = 0, r = 0, x = 0, t = 0;
    HIP_TRY(h, hipEventElapsedTime(&a, E[0], E[2]));     // update pass(es)
    HIP_TRY(h, hipEventElapsedTime(&r, E[5], E[3]));     // reduce, resample, publication
    HIP_TRY(h, hipEventElapsedTime(&t, E[0], E[3]));     // the scan on the device
    // the algorithmic byte model (include/fs2.h fs2_profile)
    const uint64_t n = (uint64_t)h->n, nblk = (uint64_t)h->nblocks();
    const uint64_t box_rows = h->row_boxes(h->cur) ? (uint64_t)h->rows : 0ull;
    const bool filt = h->cfg.gate_filter != 0;
    const uint64_t cand_bytes = filt ? sizeof(Desc) * st.groups + 128ull * st.opened + 8ull * st.words +
                                           8ull * n * p.passes + 4ull * box_rows * nblk
                                     : 0ull;
    const uint64_t upd_fixed = p.fixed_bytes + (filt ? 4ull * n * p.passes : 0ull) + 8ull * n * (uint64_t)p.m;
    const uint64_t exact_bytes = upd_fixed + (filt ? 8ull * st.words : 0ull) + 48ull * st.candidates +
                                 (64ull + sizeof(Desc)) * st.written + (2ull * kPageBytes + sizeof(Desc)) * st.cow_pages +
                                 8ull * box_rows * nblk;
    if (filt && p.m <= kMaxM) {
        // k_candidates and, one pass, k_update alone
        HIP_TRY(h, hipEventElapsedTime(&f, E[0], E[1]));
        HIP_TRY(h, hipEventElapsedTime(&x, E[4], E[2]));
        h->prof.exact_launches += 1;
        h->prof.exact_ms += x;
        h->prof.filter_launches += 1;
        h->prof.filter_ms += f;
        h->prof.filter_bytes += cand_bytes;
        h->prof.model_groups += st.groups;
        h->prof.model_opened += st.opened;
        h->prof.model_words += st.words;
        h->prof.model_candidates += st.candidates;
        h->prof.model_written += st.written;
        h->prof.model_cow += st.cow_pages;
        h->prof.model_fixed_bytes += upd_fixed;
        h->prof.model_box_bytes += 12ull * box_rows * nblk;
    }
    h->prof.scans += 1;
    h->prof.update_launches += p.passes;
    h->prof.update_ms += a;
    h->prof.reduce_ms += r;
    h->prof.scan_ms += t;
    h->prof.update_bytes += cand_bytes + exact_bytes;
    if (st.resampled)
        // page-table rows (read + write per page of every output) + scalar gather +
        // plan arrays
        h->prof.resample_bytes += 2ull * sizeof(Desc) * (st.resample_slots / kPageSlots) +
                                  2ull * 36ull * (uint64_t)h->n + 40ull * (uint64_t)h->n;
    return FS2_OK;
}

// Wait for k_publish's flag: spin for up to 50 ms (a scan at config 3 takes
// under 1 ms), then fall back to a stream sync, which also reports a fault.
static int wait_flag(fs2_handle *h, unsigned long long seq) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
        if (__atomic_load_n(h->pub_flag, __ATOMIC_ACQUIRE) == seq) return FS2_OK;
        if ((it & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
        __builtin_ia32_pause();
    }
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (__atomic_load_n(h->pub_flag, __ATOMIC_ACQUIRE) != seq)
        return set_err(&h->err, FS2_ERR_HIP, "scan statistics were not published");
    return FS2_OK;
}

// The tail of a scan whose update pass is enqueued: normalise, N_eff, estimate,
// the resample when the rule fires, the publication (fast_slam_2.py:161-223).  In a
// plain submit right after the update pass; for the second of two outstanding
// scans when the first is waited for (h->cur is then the set its update used).
static int enqueue_tail(fs2_handle *h, const fs2_handle::TailCtx &t) {
    int rc = FS2_OK;
    const int cur = h->cur;
    hipStream_t s = h->stream;
    const int G = h->cfg.world_size;
    const bool sh = h->tp != nullptr;
    const int red = h->reduce();
    const bool seq = red == FS2_REDUCE_SEQUENTIAL && !sh;
    const bool exact = red == FS2_REDUCE_EXACT;
    const double flip_margin = (red == FS2_REDUCE_PARALLEL) ? std::ldexp(2.0 * (double)h->n_global + 64.0, -53) : 0.0;
    const bool prof = t.prof;
    hipEvent_t *E = h->ev.e[t.evset];
    // ---- normalise, N_eff, estimate ----
    ReduceParams rp{};
    rp.n = h->n;
    rp.n_global = h->n_global;
    rp.gidx0 = h->first;
    rp.w = h->w[cur];
    rp.cnt = h->cnt[cur];
    rp.x = h->x[cur]; rp.y = h->y[cur]; rp.yaw = h->yaw[cur];
    rp.wpart = h->wpart;
    rp.cpart = h->cpart + (size_t)t.par * kNumCounters * (size_t)h->nblocks();
    rp.nwpart = (int32_t)h->nblocks();
    rp.part_sq = h->part_sq;
    rp.part_best_w = h->part_best_w;
    rp.part_best_i = h->part_best_i;
    rp.part_maxcnt = h->part_maxcnt;
    rp.nparts = (int32_t)h->nblocks();
    rp.floor = h->cfg.weight_floor;
    rp.sequential = seq ? 1 : 0;
    rp.exact = exact ? 1 : 0;
    rp.np_part = h->np_part;
    rp.n_np = (int32_t)np_sumsq_chunks(h->n);
    rp.flip_margin = flip_margin;
    rp.part_w = exact ? h->part_w : nullptr;
    rp.np_leaf = exact ? h->np_leaf : nullptr;
    // exact mode on one GPU: normalise and numpy's chunk trees in one pass
    // (k_normalize_chunks)
    rp.chunked = (exact && !sh) ? 1 : 0;
    if (rp.chunked) rp.nparts = normalize_chunk_parts(h->n);
    rp.part_pose = h->part_pose;
    rp.np_tail = exact ? h->np_tail : nullptr;
    rp.u0_host = t.has_u0 ? h->u0_dev : nullptr;
    rp.seed = h->cfg.seed;
    rp.scan = h->scan;
    rp.stats = h->stats_dev;
    rp.world = G;
    rp.rank = h->cfg.rank;
    rp.shard = h->shard;
    std::memcpy(rp.rank_of, h->rank_of, sizeof rp.rank_of);
    rp.rec = h->rec;
    rp.recs = sh ? h->recs : h->rec;
    rp.totals = h->totals;
    rp.want_collect = t.want_collect;

    const int nxt = 1 - cur;
    ResampleParams rs{};
    rs.n = h->n;
    rs.N = h->n_global;
    rs.a = h->first;
    rs.ao = h->first;        // the outputs stay in this shard unless exchange_particles moves it
    rs.keep = h->shard;
    // a rank that may take another shard learns which one after the plan counts:
    // its first k_ranges stores the ranges only, the outputs are filled after
    rs.ranges_mode = (sh && h->follow) ? 1 : 3;
    rs.w = h->w[cur];
    rs.c = h->cbuf;
    rs.bsum = h->bsum;
    rs.nblk = (int32_t)((h->n + 1023) / 1024);
    rs.mlo = h->mlo;
    rs.mhi = h->mhi;
    rs.out_src = h->out_src;
    rs.runs = h->runs;
    rs.runs_n = h->runs_n;
    rs.x = h->x[cur]; rs.y = h->y[cur]; rs.yaw = h->yaw[cur]; rs.cnt = h->cnt[cur];
    rs.ox = h->x[nxt]; rs.oy = h->y[nxt]; rs.oyaw = h->yaw[nxt]; rs.ow = h->w[nxt]; rs.ocnt = h->cnt[nxt];
    rs.map = h->map();
    rs.opt = h->pt[nxt];
    rs.obbox = h->row_boxes(nxt);
    rs.rank_d = h->rank_d;
    rs.rank_e = h->rank_e;
    rs.iblk = h->iblk;
    rs.part_best_w = h->part_best_w;
    rs.part_best_i = h->part_best_i;
    rs.part_slots = h->part_slots;
    rs.stats = h->stats_dev;
    rs.rec = h->rec;
    rs.flip_margin = flip_margin;
    rs.use_chain = exact ? 1 : 0;
    rs.refs = h->refs ? 1 : 0;
    if (h->refs && h->xt_key) {
        rs.tkey = h->xt_key;
        rs.tcap = h->xt_cap;
        rs.tepoch = ++h->loc_epoch;
    }
    rs.chain = ChainView{h->uinfo, h->ugl, h->uol, h->bpd, h->bpc, h->seql, h->sout, h->uel, h->bpe};
    rs.gen = sh ? nullptr : h->gen_dev;      // (one GPU: k_tail_single bumps it on a resample)

    // weight total over all ranks (fast_slam_2.py:166).  Exact: Python's sum (in
    // particle order) from the update pass's block sums, the chain's units also
    // folding the update counters (k_wsum's other job)
    const bool xsh = sh && exact;            // exact orders across shards
    if (prof && exact && !xsh && h->n <= 0) HIP_TRY(h, hipEventRecord(E[5], s));   // launch_chain records nothing
    if (exact && !xsh) {
        ChainParams cp = h->chain(h->w[cur], h->wpart, nullptr, &h->stats_dev->total, false);
        cp.cpart = h->cpart + (size_t)t.par * kNumCounters * (size_t)h->nblocks();
        cp.ncpart = (int32_t)h->nblocks();
        cp.cstats = h->stats_dev;
        HIP_TRY(h, launch_chain(cp, s, prof ? E[5] : nullptr));
    } else {
        HIP_TRY(h, launch_wsum(rp, s, prof ? E[5] : nullptr));
    }
    // a sharded rank's chain ops (xsh): its units classified against the tree
    // prefix of the shards before it, exported as exact adds
    auto chain_ops = [&](ChainParams cp, const double *est) -> int {
        cp.chain_first = h->shard == 0 ? 1 : 0;
        cp.force_list0 = 1;
        cp.est_base = est;
        cp.ops_out = h->dch_send;
        cp.uop = h->uop;
        HIP_TRY(h, launch_chain_export(cp, s));
        CommTimer ct(h);
        return h->tp->allgather(h->dch_send, h->dch_recv, sizeof(ChainSummary), s, &h->err);
    };
    if (sh) {
        {
            CommTimer ct(h);
            rc = h->tp->allgather(&h->stats_dev->total, h->totals, sizeof(double), s, &h->err);
        }
        if (rc) return rc;
        rp.est_base = xsh ? h->est_base : nullptr;
        HIP_TRY(h, launch_global_total(rp, s));
        if (xsh) {
            // Python's sum over the global order: every rank folds all shards' ops
            rc = chain_ops(h->chain(h->w[cur], h->wpart, nullptr, nullptr, false), h->est_base);
            if (rc) return rc;
            HIP_TRY(h, launch_chain_fold(h->dch_recv, G, h->shard, h->rank_of, &h->stats_dev->total, nullptr,
                                         h->stats_dev, s));
        }
    }
    if (xsh) {
        // normalise (tree partials for the estimates), numpy's Sigma w'^2 over the
        // global chunks, this rank's record, all records, the decision
        rp.exact = 0;
        rp.np_leaf = nullptr;
        rp.part_w = h->part_w;
        rp.t_from_parts = 1;
        rp.rec = &h->recx->base;
        HIP_TRY(h, launch_normalize(rp, s));
        HIP_TRY(h, launch_np_shard(h->w[cur], h->n, h->first, h->n_global, h->np_tail_g, h->recx, s));
    } else {
        // normalise (:161-175), local prefix of the normalised weights, this rank's record
        HIP_TRY(h, rp.chunked ? launch_normalize_chunks(rp, s) : launch_normalize(rp, s));
        // sharded ranks need their prefix end in the record; one GPU needs the
        // prefix only when the rule fires (computed below, kernels exit otherwise)
        if (sh) HIP_TRY(h, launch_prefix(rs, seq ? 1 : 0, s));
    }
    // one GPU: k_finalize publishes a scan whose rule did not fire, before the
    // lazy resample kernels (they run while the host returns)
    const unsigned long long pseq = ++h->pub_seq;
    if (!sh) {
        rp.pub_host = h->pub_stats_dev;
        rp.pub_flag = h->pub_flag_dev;
        rp.pub_seq = pseq;
    }
    HIP_TRY(h, rp.chunked ? launch_finalize_chunked(rp, s) : launch_finalize(rp, s));
    if (sh) {
        {
            CommTimer ct(h);
            rc = xsh ? h->tp->allgather(h->recx, h->recxs, sizeof(RankRecordX), s, &h->err)
                     : h->tp->allgather(h->rec, h->recs, sizeof(RankRecord), s, &h->err);
        }
        if (rc) return rc;
    }
    // N_eff (:212-223), resample rule (:62), estimate (:201-210), u0 (:183); on
    // one GPU k_finalize did this already
    if (sh) HIP_TRY(h, xsh ? launch_global_finalize_x(rp, h->recxs, h->np_tail_g, s) : launch_global_finalize(rp, s));
    if (!sh) {
        rs.lazy = 1;
        if (exact)   // the resample's running sum (fast_slam_2.py:184-193), bit-exact
            HIP_TRY(h, launch_chain(h->chain(h->w[cur], h->part_w, h->cbuf, nullptr, true), s));
        else
            HIP_TRY(h, launch_prefix(rs, seq ? 1 : 0, s));
    }

    // ---- low-variance resample (:177-199); on one GPU the kernels exit unless the
    // rule fired, sharded ranks learn the decision first (sizes of the transfers) ----
    bool run_resample = true;
    if (sh) {
        rc = post_and_wait(h, false);
        if (rc) return rc;
        run_resample = posted_stats(h).resampled != 0;
    }
    if (run_resample) {
        if (xsh) {
            // the running sum over the global order (fast_slam_2.py:184-193): every
            // rank folds all shards' ops for the exact value before its first
            // particle, then walks its own units from there
            ChainParams cp = h->chain(h->w[cur], h->part_w, h->cbuf, nullptr, false);
            rc = chain_ops(cp, &h->stats_dev->offset);
            if (rc) return rc;
            HIP_TRY(h, launch_chain_fold(h->dch_recv, G, h->shard, h->rank_of, nullptr, &h->stats_dev->offset,
                                         h->stats_dev, s));
            cp.chain_first = h->shard == 0 ? 1 : 0;
            cp.force_list0 = 1;
            cp.s_entry = &h->stats_dev->offset;
            HIP_TRY(h, launch_chain_walk_from(cp, s));
        }
        // one GPU: the post-resample estimate comes from the sources (k_ranges), so the
        // scan is published before the gather -- the host returns and enqueues the
        // next scan while the maps are copied, instead of after
        if (!sh) {
            rs.est_early = 1;
            rs.go = h->go_dev;
            rs.go_seq = pseq;
        }
        // every local output is written below: the output ranges of the local
        // sources (k_ranges) and of the received ones (k_scatter_recv) partition them
        HIP_TRY(h, launch_resample_ranges(rs, s, sh));     // (one GPU: k_tail_single fills the runs)
        if (!sh)
            HIP_TRY(h, launch_tail_single(rs, rp, h->pub_stats_dev, h->pub_flag_dev, pseq, s, nullptr));
        if (sh) {
            rc = exchange_particles(h, rs);
            if (rc) return rc;
            // received maps can be longer than every local one: rows for the
            // largest map on any rank (k_global_finalize) before unpacking them
            if (posted_stats(h).max_count > h->cap) scan_alloc(h, "scan_alloc rows (slots M)", (size_t)posted_stats(h).max_count << 20);
            rc = grow_rows(h, posted_stats(h).max_count);
            if (rc) return rc;
            rs.opt = h->pt[nxt];
            rs.obbox = h->row_boxes(nxt);
            // fresh pages and records for the received distinct pages: page u ->
            // page freel[base + u], its slot j -> record rfreel[rbase + 8 u + j]
            rc = reserve_recs(h, h->u_recv * kPageSlots, &rs.alloc);
            if (rc) return rc;
            rc = reserve_pages(h, h->u_recv, &rs.alloc);
            if (rc) return rc;
            rs.map = h->map();
            // received rows and pages: sized for every local output's whole row at
            // creation and with every row growth (recv_bufs), so these never fire
            // unless n_recv * rows overflowed that (counted in scan_allocs)
            const size_t rbytes = sizeof(XDesc) * (size_t)std::max<int64_t>((int64_t)h->n_recv * h->rows, 1);
            const size_t ubytes = sizeof(XDesc) * (size_t)std::max<int64_t>(h->u_recv, 1);
            if (rbytes > h->rdesc_cap || ubytes > h->udesc_cap) {
                scan_alloc(h, "scan_alloc recv rows (MiB)", std::max(rbytes, ubytes));
                rc = recv_bufs(h, std::max(rbytes, ubytes));
                if (rc) return rc;
            }
            rs.udesc = h->udesc;
            rs.rdesc = h->rdesc;
        }
        HIP_TRY(h, launch_resample_apply(rs, sh, s));
        if (sh) {
            {
                CommTimer ct(h);
                rc = h->tp->allgather(h->rec, h->recs, sizeof(RankRecord), s, &h->err);
            }
            if (rc) return rc;
            HIP_TRY(h, launch_global_best(rp, s));
        }
    }

    // publish the stats to host memory and spin on the flag: a stream sync's
    // wake-up and a copy launch cost more than the whole reduction phase (one
    // GPU: together with the post-resample estimate, in one launch)
    if (sh)
        HIP_TRY(h, launch_publish(h->stats_dev, h->pub_stats_dev, h->pub_flag_dev, pseq, s, prof ? E[3] : nullptr));
    else if (prof)
        HIP_TRY(h, hipEventRecord(E[3], s));   // (the tail's end: after the gather, published before it)
    h->stats_clean = true;
    h->pending.on = true;
    h->pending.seq = pseq;
    h->pending.prof = prof;
    h->pending.passes = t.passes;
    h->pending.m = t.M;
    h->pending.fixed_bytes = t.fixed_bytes;
    return FS2_OK;
}


static int complete_oldest(fs2_handle *h, double out_pose[3], fs2_iter_stats *stats);
static int mt_finish(fs2_handle *h);

int fs2_iterate_submit(fs2_handle *h, double rotation, double translation, const double *meas,
                       const double *observed, int32_t M, const double *noise, const double *u0) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    if ((h->stash.on ? 1 : 0) + (h->pending.on ? 1 : 0) >= 2)
        return set_err(&h->err, FS2_ERR_STATE, "two scans are outstanding: fs2_iterate_wait for the oldest first");
    if (M < 0 || (M > 0 && !meas)) return set_err(&h->err, FS2_ERR_ARG, "bad measurements (M=%d)", M);
    // draws of fs2_mt_draw (numpy's stream, made on the device) stand in for noise /
    // u0; a draw is consumed by this call whatever happens below
    const bool drawn = h->mt.armed || h->mt.deferred;
    h->mt.armed = false;
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    // a deferred draw ends between k_candidates and k_update below, or on the way out
    // (its outputs are written whatever this call returns)
    struct DrawEnd {
        fs2_handle *h;
        ~DrawEnd() {
            if (h->mt.deferred) {
                mt_finish(h);
                h->mt.armed = false;
            }
        }
    } draw_end{h};
    if (drawn && (noise || u0))
        return set_err(&h->err, FS2_ERR_ARG, "fs2_iterate: noise / u0 given after fs2_mt_draw");
    int rc;
    // A scan outstanding: it is completed here and its results wait for
    // fs2_iterate_wait.  (Round 5 enqueued this scan's update pass behind the
    // outstanding one's tail when nothing needed its outcome first, the two scans in
    // flight reading their buffer set on the device; measured no faster in order --
    // profiles/r05_ab_pipelined.txt -- and removed in round 6.)
    if (h->pending.on) {
        h->stash.rc = complete_oldest(h, h->stash.pose, &h->stash.st);
        h->stash.on = true;
        if (h->stash.rc)
            return set_err(&h->err, FS2_ERR_STATE, "the outstanding scan failed (fs2_iterate_wait reports it)");
    }
    const int par = (int)(h->submitted & 1u);
    const uint64_t scan_id = h->scan;
    if (h->refs && !h->refs_shared) {
        rc = share_pools(h, true);
        if (rc) return rc;
    }
    bool collected = false;
    if (h->refs_shared && h->collect_next) {
        // page_refs: some rank's pools ran short in the last scan (every rank read the
        // same records, so every rank collects -- and grows -- here, together)
        if (h->collect_next & 6) {
            rc = regrow_collective(h, (h->collect_next & 2) ? 1 : 0, (h->collect_next & 4) ? 1 : 0);
            if (rc) return rc;
        }
        rc = collect_collective(h);
        if (rc) return rc;
        h->collect_next = 0;
        collected = true;
    }
    if (h->refs_shared && h->room_check) {
        // after a resample (every rank knows it resampled) the remote rows this scan
        // may localise are new: the ranks agree, before any localisation, whether
        // some rank lacks room for them and this scan's reservations -- then every
        // rank collects, and grows what is still short, together
        h->room_check = false;
        const int64_t Mx = std::max<int64_t>(M, 1);
        auto short_bits = [&]() -> uint8_t {
            const int64_t pneed = Mx * h->n + h->remote_bound();
            const int64_t rneed = Mx * h->n + (int64_t)kPageSlots * h->remote_bound();
            return (uint8_t)((h->nfree - h->cursor < 2 * pneed ? 1 : 0) | (h->rnfree - h->rcursor < 2 * rneed ? 2 : 0));
        };
        auto any_short = [&](uint8_t mine, uint8_t *all_or) -> int {
            uint8_t all[kMaxRanks] = {};
            HIP_TRY(h, hipMemsetAsync(h->ep_dev, mine, 1, h->stream));
            {
                CommTimer ct(h);
                const int rc2 = h->tp->allgather(h->ep_dev, h->epochs_dev, 1, h->stream, &h->err);
                if (rc2) return rc2;
            }
            HIP_TRY(h, hipMemcpyAsync(all, h->epochs_dev, (size_t)h->cfg.world_size, hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(h, hipStreamSynchronize(h->stream));
            if (int rc2 = h->tp->status(&h->err)) return rc2;
            *all_or = 0;
            for (int q = 0; q < h->cfg.world_size; ++q) *all_or |= all[q];
            return FS2_OK;
        };
        uint8_t any = 0;
        trace(h, "room check remote pages (K)", (int)(h->remote_bound() >> 10));
        rc = any_short(short_bits(), &any);
        trace(h, "room short", any);
        if (rc) return rc;
        if (any && !collected) {
            rc = collect_collective(h);
            if (rc) return rc;
            collected = true;
            rc = any_short(short_bits(), &any);
            if (rc) return rc;
        }
        if (any) {
            const uint8_t mine = short_bits();
            const int64_t pneed = Mx * h->n + h->remote_bound();
            const int64_t rneed = Mx * h->n + (int64_t)kPageSlots * h->remote_bound();
            rc = regrow_collective(h, (mine & 1) ? h->npool - (h->nfree - h->cursor) + 3 * pneed : 0,
                                   (mine & 2) ? h->nrecs - (h->rnfree - h->rcursor) + 3 * rneed : 0);
            if (rc) return rc;
        }
    }
    trace(h, "submit", (int)scan_id);
    rc = grow_rows(h, h->cnt_upper + M);
    if (rc) return rc;
    const int cur = h->cur;
    hipStream_t s = h->stream;
    const bool sh = h->tp != nullptr;             // sharded path (G > 1, or forced for testing)
    const bool prof = h->profiling && (h->prof_tick++ % (uint64_t)h->prof_period) == 0;

    // (pinned staging by scan parity: the outstanding scan's copies may not have run)
    if (noise) {
        double *pin = h->noise_pin + (size_t)par * (size_t)h->n;
        std::memcpy(pin, noise, sizeof(double) * h->n);
        HIP_TRY(h, hipMemcpyAsync(h->noise_dev, pin, sizeof(double) * h->n, hipMemcpyHostToDevice, s));
    }
    if (u0) {
        double *pin = h->u0_pin + par;
        *pin = *u0;
        HIP_TRY(h, hipMemcpyAsync(h->u0_dev, pin, 8, hipMemcpyHostToDevice, s));
    }
    if (h->cfg.record_assoc && (int64_t)M * h->n > h->assoc_cap) {
        HIP_TRY(h, hipStreamSynchronize(s));
        hipFree(h->assoc_dev);
        h->assoc_dev = nullptr;
        HIP_TRY(h, hipMalloc(&h->assoc_dev, sizeof(int32_t) * (size_t)M * h->n));
        h->assoc_cap = (int64_t)M * h->n;
    }
    // the last scan's k_publish zeroed the stats; anything else (first scan, an
    // error return) leaves them to be cleared here
    if (!h->stats_clean) HIP_TRY(h, hipMemsetAsync(h->stats_dev, 0, sizeof(DevStats), s));
    h->stats_clean = false;
    if (prof && h->ev.used == kProfSets) {   // pool used up: fold (the scans are long complete)
        const int rc0 = fold_profile(h);
        if (rc0) return rc0;
    }
    // (event sets are taken by profiled scans only: the outstanding one's if it was)
    const int evset = h->ev.used;
    hipEvent_t *E = h->ev.e[evset];

    // ---- fused update passes (move in the first) ----
    UpdateParams up{};
    up.n = h->n;
    up.nblk = h->nblocks();
    up.blk0 = 0;
    up.blk1 = up.nblk;
    up.gidx0 = h->first;
    up.x = h->x[cur]; up.y = h->y[cur]; up.yaw = h->yaw[cur]; up.w = h->w[cur]; up.cnt = h->cnt[cur];
    up.map = h->map();
    up.noise = (noise || drawn) ? h->noise_dev : nullptr;
    up.seed = h->cfg.seed;
    up.scan = scan_id;
    up.sigma = (rotation != 0) ? h->cfg.rotation_noise : h->cfg.translation_noise;
    up.rotation = rotation;
    up.translation = translation;
    up.gate2 = h->gate2;
    // gate2 / (1 - 2^-18) rounded up: slack for the fp32 rounding in gate_reject_fast
    up.gate2f = std::isinf(h->gate2) ? INFINITY
                                     : std::nextafter((float)(h->gate2 / (1.0 - 0x1p-18)), INFINITY);
    up.filter = h->cfg.gate_filter ? 1 : 0;
    up.cand = h->cand;
    up.ncand = h->ncand;
    std::memcpy(up.R, h->cfg.measurement_noise, sizeof up.R);
    std::memcpy(up.init_cov, h->cfg.init_landmark_cov, sizeof up.init_cov);
    up.assoc = h->cfg.record_assoc ? h->assoc_dev : nullptr;
    up.wpart = h->wpart;
    up.cpart = h->cpart + (size_t)par * kNumCounters * (size_t)h->nblocks();
    up.stats = h->stats_dev;
    up.slb_pass = h->slb_pass;
    if (!sh) {                  // one GPU: the buffer set is taken on the device (BufSet)
        up.gen = h->gen_dev;
        up.sets = h->sets_dev;
    }
    // page_refs: this scan may ask for a collective collection before the next one
    // (its pools' room after this scan's reservations and localisations, at most
    // the remote row entries, below twice as much again)
    int32_t want_collect = 0;
    if (h->refs) {              // (also before references cross: this scan's resample may send them)
        const int64_t pneed = (int64_t)std::max(M, 1) * h->n + h->remote_bound();
        const int64_t rneed = (int64_t)std::max(M, 1) * h->n + (int64_t)kPageSlots * h->remote_bound();
        const bool plow = h->nfree - h->cursor < 3 * pneed, rlow = h->rnfree - h->rcursor < 3 * rneed;
        want_collect = (plow || rlow) ? 1 : 0;
        // still short right after a collective collection: every rank grows next scan
        if (collected && plow) want_collect |= 2;
        if (collected && rlow) want_collect |= 4;
    }
    int passes = 0;
    uint64_t fixed_bytes = 0;
    for (int32_t k0 = 0; k0 < std::max(M, 1); k0 += kMaxM) {
        const int32_t m = std::min(kMaxM, M - k0);
        up.do_move = (k0 == 0);
        // the motion sample in the candidate pass unless a deferred numpy draw ends
        // only after it (mt_finish below) or no candidate pass runs (no gate filter)
#ifdef FS2_AB_MOVE_IN_UPDATE
        up.move_cand = 0;
#else
        up.move_cand = (up.do_move && up.filter && !h->mt.deferred) ? 1 : 0;
#endif
        up.k0 = k0;
        up.m = std::max(m, 0);
        up.last_pass = (k0 + kMaxM >= M);
        for (int k = 0; k < kMaxM; ++k) {
            if (k < up.m) {
                const double d = meas[2 * (k0 + k)], b = meas[2 * (k0 + k) + 1];
                up.meas.d[k] = d;
                up.meas.b[k] = b;
                up.meas.ox[k] = observed ? observed[2 * (k0 + k)] : d * std::cos(b);
                up.meas.oy[k] = observed ? observed[2 * (k0 + k) + 1] : d * std::sin(b);
            } else {
                up.meas.d[k] = up.meas.b[k] = up.meas.ox[k] = up.meas.oy[k] = 0.0;
            }
            // fp32 observed point for the gate mirror and a bound on its rounding
            const double ox = up.meas.ox[k], oy = up.meas.oy[k];
            up.meas.fx[k] = (float)ox;
            up.meas.fy[k] = (float)oy;
            const double e = std::max(std::fabs(ox - (double)up.meas.fx[k]),
                                      std::fabs(oy - (double)up.meas.fy[k]));
            up.meas.fe[k] = std::isfinite(e) ? std::nextafter((float)e, INFINITY) : INFINITY;
        }
        rc = reserve_recs(h, (int64_t)up.m * h->n, &up.alloc);
        if (rc) return rc;
        rc = reserve_pages(h, (int64_t)up.m * h->n, &up.alloc);
        if (rc) return rc;
        up.map = h->map();
        const bool first = k0 == 0, last = up.last_pass != 0;
        const bool cand = up.filter && up.blk1 > up.blk0;
        if (h->refs_shared && h->remote_rows > 0 && up.blk1 > up.blk0) {
            // page_refs: the remote pages this pass could read, localised first (from
            // the free lists' tails, clear of every reservation this scan makes; a
            // tail too short fails the scan loudly, fs2.h error_flags bit 3)
            const int64_t left = (int64_t)std::max(M - k0 - up.m, 0) * h->n;   // later passes' reservations
            LocalizeParams lp{};
            lp.pcap = h->nfree - h->cursor - left;
            lp.rcap = h->rnfree - h->rcursor - left;
            lp.map = up.map;
            lp.cnt = up.cnt;
            lp.n = h->n;
            lp.nblk = up.nblk;
            lp.m = up.m;
            lp.gate2f = up.gate2f;
            lp.meas = up.meas;
            lp.freel = h->freel;
            lp.ftail = h->nfree;
            lp.rfreel = h->rfreel;
            lp.rtail = h->rnfree;
            lp.stats = h->stats_dev;
            // one copy per distinct remote page: the page-dedup table the page
            // transfer would use (sized for every row of the shard, xfer_bufs), keys
            // tagged with this pass's epoch so it is never cleared
            lp.key = h->xt_key;
            lp.val = h->xt_uidx;
            lp.cap = h->xt_cap;
            lp.epoch = ++h->loc_epoch;
            HIP_TRY(h, launch_localize(lp, s));
        }
        // a shard without particles launches nothing: its profiled intervals are
        // recorded empty here (fold_one reads every event of the set)
        if (prof && first && up.blk1 <= up.blk0)
            for (int k : {0, 1, 4}) HIP_TRY(h, hipEventRecord(E[k], s));
        HIP_TRY(h, launch_candidates(up, s, (prof && first) ? E[0] : nullptr, (prof && first) ? E[1] : nullptr));
        if (first && h->mt.deferred) {     // the draw's host half while k_candidates runs
            rc = mt_finish(h);
            if (rc) return rc;
            h->mt.armed = false;
        }
        HIP_TRY(h, launch_update(up, s, (prof && first) ? (cand ? E[4] : E[0]) : nullptr,
                                 (prof && last) ? E[2] : nullptr));
        if (prof && last && up.blk1 <= up.blk0) HIP_TRY(h, hipEventRecord(E[2], s));
        ++passes;
        // pose/weight/count read + weight/count write; pose write on the move pass
        fixed_bytes += (uint64_t)h->n * (32 + 4 + 8 + 4 + (up.do_move ? 24 : 0));
        if (up.do_move && (noise || drawn)) fixed_bytes += (uint64_t)h->n * 8;
        if (up.assoc) fixed_bytes += (uint64_t)h->n * 4 * up.m;
    }
    h->submitted += 1;

    fs2_handle::TailCtx tc;
    tc.M = M;
    tc.passes = passes;
    tc.fixed_bytes = fixed_bytes;
    tc.prof = prof;
    tc.evset = evset;
    tc.want_collect = want_collect;
    tc.has_u0 = (u0 || drawn);
    tc.par = par;
    return enqueue_tail(h, tc);
}

// The oldest outstanding scan: its publication, the host's bookkeeping (which set
// is current, reservations, profile), its pose and statistics.
static int complete_oldest(fs2_handle *h, double out_pose[3], fs2_iter_stats *stats) {
    h->pending.on = false;
    const int M = h->pending.m;
    int rc = wait_flag(h, h->pending.seq);
    if (rc) return rc;
    // a stream-ordered transport reports a failed collective only now
    if (h->tp && (rc = h->tp->status(&h->err))) return rc;
    const DevStats &st = *h->pub_stats;
    if (h->refs_shared) {
        // page_refs: the free lists' tails the localisations took; the remote row
        // entries left (recounted by a resample's gather); a collective collection next?
        h->nfree -= (int64_t)st.loc_pages;
        h->rnfree -= (int64_t)st.loc_recs;
        h->remote_rows = st.resampled ? (int64_t)st.remote_rows
                                      : std::max<int64_t>(0, h->remote_rows - (int64_t)st.loc_rows);
        if (st.resampled) h->remote_pages = (int64_t)st.remote_pages;
        h->collect_next = st.collect_next;
        if (h->profiling) {
            h->prof.localized_pages += st.loc_pages;
        }
    }
    if (st.resampled) h->cur = 1 - h->cur;
    if (st.resampled && h->refs_shared) h->room_check = true;   // new remote rows: agree on room next scan
    h->appends_since_rcollect += (int64_t)st.appends;
    if (st.resampled) h->rcollect_exact = false;     // dropped particles' records: no bound
    h->cnt_upper = st.max_count;
    h->last_m = M;
    h->scan += 1;
    if (h->profiling) h->prof.sent_pages_repeat += st.repeat_pages;
    if (h->pending.prof) {
        ProfScan &p = h->ev.scan[h->ev.used++];
        p.st = st;
        p.passes = h->pending.passes;
        p.m = M;
        p.fixed_bytes = h->pending.fixed_bytes;
    }
    if (out_pose) {
        out_pose[0] = st.pose[0];
        out_pose[1] = st.pose[1];
        out_pose[2] = st.pose[2];
    }
    if (stats) {
        stats->resampled = st.resampled;
        stats->max_count = st.max_count;
        stats->n_eff = st.n_eff;
        stats->total_weight = st.total;
        stats->best_index = st.best_index;
        stats->slots_visited = st.visited;
        stats->candidates = st.candidates;
        stats->hits = st.hits;
        stats->appends = st.appends;
        stats->slots_written = st.written;
        stats->ambiguous = st.ambiguous;
        stats->resample_slots = st.resample_slots;
        stats->error_flags = st.error_flags;
        stats->reduce_ambiguous = (int32_t)std::min<unsigned long long>(st.reduce_amb, INT32_MAX);
        stats->cow_pages = st.cow_pages;
        stats->new_pages = st.new_pages;
        stats->collections = h->collections;
        stats->pool_pages = (uint64_t)h->npool;
        stats->pool_records = (uint64_t)h->nrecs;
        stats->pool_copies = h->vm_fallbacks;
        stats->pages_opened = st.opened;
        stats->reference_visits = st.ref_visits;
    }
    if (st.error_flags & 1)
        return set_err(&h->err, FS2_ERR_LINALG, "Singular matrix (landmark or observation covariance)");
    if ((st.error_flags & 4) && h->cfg.reduce_mode == FS2_REDUCE_EXACT)
        return set_err(&h->err, FS2_ERR_STATE,
                       "sharded exact-order reduction incomplete (chain ops overflow or numpy chunk edges): "
                       "the scan used the tree estimate, not the reference's summation order");
    if (st.error_flags & 8) return refs_short(h, "page or record");
    return FS2_OK;
}

int fs2_iterate_wait(fs2_handle *h, double out_pose[3], fs2_iter_stats *stats) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    if (h->stash.on) {                 // completed by a submit that had to wait for it
        h->stash.on = false;
        if (out_pose) std::memcpy(out_pose, h->stash.pose, sizeof h->stash.pose);
        if (stats) *stats = h->stash.st;
        return h->stash.rc;
    }
    if (!h->pending.on) return set_err(&h->err, FS2_ERR_STATE, "no submitted scan to wait for");
    fs2_iter_stats st_local{};
    return complete_oldest(h, out_pose, stats ? stats : &st_local);
}

int fs2_iterate(fs2_handle *h, double rotation, double translation, const double *meas,
                const double *observed, int32_t M, const double *noise, const double *u0,
                double out_pose[3], fs2_iter_stats *stats) {
    if (h && (h->pending.on || h->stash.on))
        return set_err(&h->err, FS2_ERR_STATE, "submitted scans are outstanding (fs2_iterate_wait first)");
    const int rc = fs2_iterate_submit(h, rotation, translation, meas, observed, M, noise, u0);
    if (rc) return rc;
    return fs2_iterate_wait(h, out_pose, stats);
}

int fs2_get_assoc(fs2_handle *h, int32_t *idx, int64_t capacity, int32_t *m_out) {
    if (!h || !idx) return set_err(h ? &h->err : nullptr, FS2_ERR_ARG, "null argument");
    if (h->pending.on) return set_err(&h->err, FS2_ERR_STATE, "a submitted scan is pending (fs2_iterate_wait first)");
    if (!h->cfg.record_assoc) return set_err(&h->err, FS2_ERR_STATE, "record_assoc is off");
    const int64_t need = (int64_t)h->last_m * h->n;
    if (capacity < need) return set_err(&h->err, FS2_ERR_ARG, "assoc buffer too small (%lld < %lld)",
                                        (long long)capacity, (long long)need);
    if (m_out) *m_out = h->last_m;
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (need) HIP_TRY(h, hipMemcpy(idx, h->assoc_dev, sizeof(int32_t) * need, hipMemcpyDeviceToHost));
    return FS2_OK;
}

static hipMemcpyKind kind_in(int32_t where) {
    return where == FS2_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
}
static hipMemcpyKind kind_out(int32_t where) {
    return where == FS2_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
}

int fs2_set_state(fs2_handle *h, int64_t first, int64_t count, const double *x, const double *y,
                  const double *yaw, const double *w, const int32_t *cnt, const double *lm,
                  int32_t lm_cap, int32_t where) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    if (h->pending.on) return set_err(&h->err, FS2_ERR_STATE, "a submitted scan is pending (fs2_iterate_wait first)");
    if (first < 0 || count < 0 || first + count > h->n)
        return set_err(&h->err, FS2_ERR_ARG, "range [%lld, %lld) outside %lld local particles",
                       (long long)first, (long long)(first + count), (long long)h->n);
    if ((cnt == nullptr) != (lm == nullptr) || (lm && lm_cap < 0))
        return set_err(&h->err, FS2_ERR_ARG, "cnt and lm must be given together");
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    {
        const int rcm = mt_finish(h);    // a pending fs2_mt_draw was made for the state replaced here
        h->mt.armed = false;
        if (rcm) return rcm;
    }
    hipStream_t s = h->stream;
    const int c = h->cur;
    HIP_TRY(h, hipStreamSynchronize(s));
    if (count == 0) return FS2_OK;
    const size_t b8 = sizeof(double) * count;
    if (x) HIP_TRY(h, copy_sync(h, h->x[c] + first, x, b8, kind_in(where)));
    if (y) HIP_TRY(h, copy_sync(h, h->y[c] + first, y, b8, kind_in(where)));
    if (yaw) HIP_TRY(h, copy_sync(h, h->yaw[c] + first, yaw, b8, kind_in(where)));
    if (w) HIP_TRY(h, copy_sync(h, h->w[c] + first, w, b8, kind_in(where)));
    if (cnt) {
        std::vector<int32_t> hc(count);
        HIP_TRY(h, hipMemcpy(hc.data(), cnt, sizeof(int32_t) * count,
                             where == FS2_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
        int32_t mx = 0;
        for (int32_t v : hc) {
            if (v < 0 || v > lm_cap) return set_err(&h->err, FS2_ERR_ARG, "count %d outside [0, %d]", v, lm_cap);
            mx = std::max(mx, v);
        }
        int rc = grow_rows(h, mx);
        if (rc) return rc;
        const int32_t rows_each = std::max(1, (mx + kPageSlots - 1) / kPageSlots);
        h->cnt_upper = std::max(h->cnt_upper, mx);
        // the collection bound (reserve_recs): the imported records are live; maps
        // replaced (imported twice, or after a scan) leave records of unknown number
        {
            int64_t used = 0;
            for (int32_t v : hc) used += v;
            h->appends_since_rcollect += used;
            if ((int64_t)h->imported.size() != h->n) h->imported.assign((size_t)h->n, 0);
            bool replaced = h->scan > 0;
            for (int64_t k = first; k < first + count; ++k) {
                replaced |= h->imported[(size_t)k] != 0;
                h->imported[(size_t)k] = 1;
            }
            if (replaced) h->rcollect_exact = false;
        }
        // stage in chunks of <= 256 MiB
        const int64_t per = (int64_t)std::max(1, lm_cap) * 6 * 8;
        const int64_t chunk = std::max<int64_t>(1, (256ll << 20) / per);
        double *stage = nullptr;
        int32_t *cstage = nullptr, *perm_dev = nullptr;
        HIP_TRY(h, hipMemsetAsync(h->ext_dev, 0, sizeof(uint32_t), s));
        HIP_TRY(h, hipMalloc(&stage, (size_t)std::min(chunk, count) * per));
        HIP_TRY(h, hipMalloc(&cstage, sizeof(int32_t) * std::min(chunk, count)));
        HIP_TRY(h, hipMalloc(&perm_dev, sizeof(int32_t) * std::max(1, lm_cap)));
        std::vector<double> rep((size_t)std::max(1, lm_cap) * 6);
        std::vector<int32_t> perm;
        int rc2 = FS2_OK;
        for (int64_t o = 0; o < count && rc2 == FS2_OK; o += chunk) {
            const int64_t k = std::min(chunk, count - o);
            hipError_t e = copy_sync(h, stage, lm + o * lm_cap * 6, (size_t)k * per, kind_in(where));
            if (e == hipSuccess) e = hipMemcpy(cstage, hc.data() + o, sizeof(int32_t) * k, hipMemcpyHostToDevice);
            // the chunk's layout, from its first map (the filter's page boxes are
            // what it serves; handles without the filter keep slot order)
            int32_t perm_len = -1;
            if (e == hipSuccess && h->cfg.gate_filter && hc[o] > kPageSlots) {
                e = hipMemcpy(rep.data(), lm + o * lm_cap * 6, sizeof(double) * 6 * (size_t)hc[o],
                              where == FS2_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost);
                if (e == hipSuccess && spatial_order(rep.data(), hc[o], perm)) {
                    perm_len = hc[o];
                    e = hipMemcpy(perm_dev, perm.data(), sizeof(int32_t) * perm_len, hipMemcpyHostToDevice);
                }
            }
            PageAlloc pa{};
            rc2 = reserve_recs(h, k * std::max(1, lm_cap), &pa);
            if (rc2) break;
            rc2 = reserve_pages(h, k * rows_each, &pa);
            if (rc2) break;
            if (e == hipSuccess)
                e = launch_import(stage, cstage, first + o, k, lm_cap, h->map(), pa, rows_each, h->cnt[c], h->ext_dev,
                                  perm_len > 0 ? perm_dev : nullptr, perm_len, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc2 = set_err(&h->err, FS2_ERR_HIP, "state import failed: %s", hipGetErrorString(e));
        }
        hipFree(stage);
        hipFree(cstage);
        hipFree(perm_dev);
        if (rc2) return rc2;
        // the summary grid covers every imported landmark with room to spare; when it
        // grows, every descriptor is re-encoded on the new grid
        uint32_t eb = 0;
        HIP_TRY(h, hipMemcpy(&eb, h->ext_dev, sizeof eb, hipMemcpyDeviceToHost));
        float ext = 0.0f;
        std::memcpy(&ext, &eb, sizeof ext);
        h->ext_seen = std::max(h->ext_seen, ext);
        // cell: the smallest multiple of 1/64 m whose 127 cells each side cover 1.25x
        // the extent (round 5 rounded it up to a power of two: up to 2x coarser boxes,
        // e.g. 1 m instead of 0.66 m at config 3, so a measurement between landmarks
        // 3 m away opened their pages through the quantisation slack alone)
#ifdef FS2_AB_POW2_CELL
        float cell = 1.0f / 64.0f;                       // (round 5, A/B)
        while (127.0f * cell < 1.25f * h->ext_seen && cell < 65536.0f) cell *= 2.0f;
#else
        float cell = (float)std::max(1.0, std::ceil(1.25 * (double)h->ext_seen / 127.0 * 64.0)) / 64.0f;
        if (!(cell < 65536.0f)) cell = 65536.0f;
#endif
        if (cell != h->frame.cell) h->frame = SumFrame{-127.0f * cell, cell, 1.0f / cell};
        // the workgroup row boxes, rebuilt from the pages on this grid
        HIP_TRY(h, launch_bbox_build(h->map(), h->cnt[c], s));
    }
    HIP_TRY(h, hipStreamSynchronize(s));
    return FS2_OK;
}

int fs2_update_known_landmarks(fs2_handle *h, double eps, double min_fraction, double *centres, int64_t cap,
                               int64_t *n_clusters) {
    if (!h || !n_clusters || (cap > 0 && !centres) || !(eps > 0.0))
        return set_err(h ? &h->err : nullptr, FS2_ERR_ARG, "fs2_update_known_landmarks: bad arguments");
    if (h->pending.on) return set_err(&h->err, FS2_ERR_STATE, "a submitted scan is pending (fs2_iterate_wait first)");
    if (h->cfg.world_size > 1)
        return set_err(&h->err, FS2_ERR_STATE, "update_known_landmarks needs every particle on one rank");
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    hipStream_t s = h->stream;
    HIP_TRY(h, hipStreamSynchronize(s));
    double2 *pts = nullptr;
    int64_t np = 0;
    HIP_TRY(h, gather_map_points(h->map(), h->cnt[h->cur], h->n, &pts, &np, s));
    // min_samples = int(len(all) / len(particles) * 0.7) (landmark_utils.py:131-132)
    const double avg = (double)np / (double)h->n_global;
    const double ms = avg * min_fraction;
    if (!(ms >= 1.0)) {
        (void)hipFree(pts);
        *n_clusters = -1;
        return FS2_OK;
    }
    int32_t status = 0;
    int64_t K = 0;
    double *dcent = nullptr;
    hipError_t e = hipMalloc(&dcent, sizeof(double) * 2 * std::max<int64_t>(cap, 1));
    if (e == hipSuccess)
        e = cluster_points(pts, np, eps, (int64_t)ms, dcent, cap, &K, nullptr, &status, s);
    if (e == hipSuccess && K <= cap && K > 0)
        e = hipMemcpy(centres, dcent, sizeof(double) * 2 * K, hipMemcpyDeviceToHost);
    (void)hipFree(pts);
    (void)hipFree(dcent);
    if (e != hipSuccess) return set_err(&h->err, FS2_ERR_HIP, "update_known_landmarks: %s", hipGetErrorString(e));
    if (status == 1) return set_err(&h->err, FS2_ERR_ARG, "Input contains NaN or infinity");
    if (status == 2) return set_err(&h->err, FS2_ERR_ARG, "landmark coordinates span too many eps-cells");
    *n_clusters = K;
    if (K > cap) return set_err(&h->err, FS2_ERR_ARG, "%lld clusters, centre buffer holds %lld", (long long)K,
                                (long long)cap);
    return FS2_OK;
}

int fs2_get_state(fs2_handle *h, int64_t first, int64_t count, double *x, double *y, double *yaw,
                  double *w, int32_t *cnt, double *lm, int32_t lm_cap, int32_t where) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    if (h->pending.on) return set_err(&h->err, FS2_ERR_STATE, "a submitted scan is pending (fs2_iterate_wait first)");
    if (first < 0 || count < 0 || first + count > h->n)
        return set_err(&h->err, FS2_ERR_ARG, "range outside local particles");
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    {
        const int rcm = mt_finish(h);    // a pending fs2_mt_draw was made for the state replaced here
        h->mt.armed = false;
        if (rcm) return rcm;
    }
    hipStream_t s = h->stream;
    const int c = h->cur;
    HIP_TRY(h, hipStreamSynchronize(s));
    if (count == 0) return FS2_OK;
    const size_t b8 = sizeof(double) * count;
    if (x) HIP_TRY(h, copy_sync(h, x, h->x[c] + first, b8, kind_out(where)));
    if (y) HIP_TRY(h, copy_sync(h, y, h->y[c] + first, b8, kind_out(where)));
    if (yaw) HIP_TRY(h, copy_sync(h, yaw, h->yaw[c] + first, b8, kind_out(where)));
    if (w) HIP_TRY(h, copy_sync(h, w, h->w[c] + first, b8, kind_out(where)));
    if (cnt) HIP_TRY(h, copy_sync(h, cnt, h->cnt[c] + first, sizeof(int32_t) * count, kind_out(where)));
    if (lm) {
        if (lm_cap < 0) return set_err(&h->err, FS2_ERR_ARG, "lm_cap < 0");
        std::vector<int32_t> hc(count);
        HIP_TRY(h, hipMemcpy(hc.data(), h->cnt[c] + first, sizeof(int32_t) * count, hipMemcpyDeviceToHost));
        for (int32_t v : hc)
            if (v > lm_cap) return set_err(&h->err, FS2_ERR_ARG, "lm_cap %d < map size %d", lm_cap, v);
        const int64_t per = (int64_t)std::max(1, lm_cap) * 6 * 8;
        const int64_t chunk = std::max<int64_t>(1, (256ll << 20) / per);
        double *stage = nullptr;
        HIP_TRY(h, hipMalloc(&stage, (size_t)std::min(chunk, count) * per));
        int rc2 = FS2_OK;
        for (int64_t o = 0; o < count && rc2 == FS2_OK; o += chunk) {
            const int64_t k = std::min(chunk, count - o);
            hipError_t e = hipMemsetAsync(stage, 0, (size_t)k * per, s);
            if (e == hipSuccess) e = launch_export(stage, first + o, k, lm_cap, h->map(), h->cnt[c], s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess) e = copy_sync(h, lm + o * lm_cap * 6, stage, (size_t)k * per, kind_out(where));
            if (e != hipSuccess) rc2 = set_err(&h->err, FS2_ERR_HIP, "state export failed: %s", hipGetErrorString(e));
        }
        hipFree(stage);
        if (rc2) return rc2;
    }
    return FS2_OK;
}

}  // extern "C"

// ------------------------------------------------------------ stateless ---

namespace {

struct Scratch {
    int device = -1;
    hipStream_t stream = nullptr;
    char *buf = nullptr;
    size_t bytes = 0;
};

std::mutex g_scratch_mu;
Scratch g_scratch[64];

int scratch_get(int32_t device, size_t bytes, Scratch **out) {
    if (device < 0 || device >= 64) return set_err(nullptr, FS2_ERR_ARG, "bad device %d", device);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev)
        return set_err(nullptr, FS2_ERR_HIP, "no HIP device %d (libfs2 has no CPU path)", device);
    Scratch &s = g_scratch[device];
    if (hipSetDevice(device) != hipSuccess) return set_err(nullptr, FS2_ERR_HIP, "hipSetDevice failed");
    if (!s.stream && hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess)
        return set_err(nullptr, FS2_ERR_HIP, "hipStreamCreate failed");
    if (s.bytes < bytes) {
        hipFree(s.buf);
        s.buf = nullptr;
        s.bytes = 0;
        if (hipMalloc(&s.buf, bytes) != hipSuccess) return set_err(nullptr, FS2_ERR_OOM, "scratch alloc failed");
        s.bytes = bytes;
    }
    s.device = device;
    *out = &s;
    return FS2_OK;
}

#define SHIP(expr)                                                                               \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return set_err(nullptr, FS2_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

size_t al16(size_t b) { return (b + 15) & ~size_t(15); }

}  // namespace

extern "C" {

int fs2_icp_batched(int32_t device, int32_t B, int32_t P, const double *src, const double *tgt,
                    int32_t max_iterations, double threshold, double *R, double *t,
                    int32_t *iterations, int32_t where) {
    if (B < 0 || P <= 0 || P > 1024 || !src || !tgt || !R || !t)
        return set_err(nullptr, FS2_ERR_ARG, "fs2_icp_batched: bad arguments (B=%d, P=%d; P <= 1024)", B, P);
    if (B == 0) return FS2_OK;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const size_t cb = al16((size_t)B * P * 16);
    const size_t need = 2 * cb + al16((size_t)B * 32) + al16((size_t)B * 16) + al16((size_t)B * 4);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, need, &sc);
    if (rc) return rc;
    char *p = sc->buf;
    double *ds = (double *)p, *dt = (double *)(p + cb), *dR = (double *)(p + 2 * cb);
    double *dT = (double *)(p + 2 * cb + al16((size_t)B * 32));
    int32_t *dI = (int32_t *)(p + 2 * cb + al16((size_t)B * 32) + al16((size_t)B * 16));
    const hipMemcpyKind kin = where == FS2_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    const hipMemcpyKind kout = where == FS2_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    SHIP(hipMemcpyAsync(ds, src, (size_t)B * P * 16, kin, sc->stream));
    SHIP(hipMemcpyAsync(dt, tgt, (size_t)B * P * 16, kin, sc->stream));
    SHIP(launch_icp(B, P, ds, dt, P, max_iterations, threshold, dR, dT, dI, sc->stream));
    SHIP(hipMemcpyAsync(R, dR, (size_t)B * 32, kout, sc->stream));
    SHIP(hipMemcpyAsync(t, dT, (size_t)B * 16, kout, sc->stream));
    if (iterations) SHIP(hipMemcpyAsync(iterations, dI, (size_t)B * 4, kout, sc->stream));
    SHIP(hipStreamSynchronize(sc->stream));
    return FS2_OK;
}

int fs2_icp(int32_t device, const double *src, int32_t n_src, const double *tgt, int32_t n_tgt,
            int32_t max_iterations, double threshold, double R[4], double t[2], int32_t *iterations) {
    if (n_src <= 0 || n_tgt <= 0 || n_src > 1024 || n_tgt > 1024 || !src || !tgt || !R || !t)
        return set_err(nullptr, FS2_ERR_ARG, "fs2_icp: bad arguments (point counts must be 1..1024)");
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const size_t bs = al16((size_t)n_src * 16), bt = al16((size_t)n_tgt * 16);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, bs + bt + 64, &sc);
    if (rc) return rc;
    double *ds = (double *)sc->buf, *dt = (double *)(sc->buf + bs);
    double *dR = (double *)(sc->buf + bs + bt), *dT = dR + 4;
    int32_t *dI = (int32_t *)(dT + 2);
    SHIP(hipMemcpyAsync(ds, src, (size_t)n_src * 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(hipMemcpyAsync(dt, tgt, (size_t)n_tgt * 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(launch_icp(1, n_src, ds, dt, n_tgt, max_iterations, threshold, dR, dT, dI, sc->stream));
    double out[6];
    int32_t it = 0;
    SHIP(hipMemcpyAsync(out, dR, 48, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipMemcpyAsync(&it, dI, 4, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipStreamSynchronize(sc->stream));
    std::memcpy(R, out, 32);
    t[0] = out[4];
    t[1] = out[5];
    if (iterations) *iterations = it;
    return FS2_OK;
}

}  // extern "C"

// --------------------------------------------------------- pipelined ICP ---
// fs2_icp_submit / fs2_icp_wait: the same alignment as fs2_icp, enqueued on a
// per-device stream of its own, so that scan s+1's alignment (one workgroup)
// runs beside scan s's filter update, which fills the rest of the GPU.  Each
// ticket owns a slot: pinned host staging for the clouds and the result, device
// buffers, and an event; the caller's arrays are copied at submit time.

namespace {

constexpr int kIcpSlots = 4;          // FS2_ICP_SLOTS in fs2.h
constexpr size_t kIcpCloud = 1024 * 16;

struct IcpSlot {
    char *host = nullptr;             // pinned: src, tgt, out (R, t, iterations)
    char *dev = nullptr;
    hipEvent_t done = nullptr;
    int64_t ticket = -1;              // outstanding ticket, -1 when free
};

struct IcpQueue {
    hipStream_t stream = nullptr;
    IcpSlot slot[kIcpSlots];
    int64_t next = 0;
};

std::mutex g_icpq_mu;
IcpQueue g_icpq[64];

int icpq_get(int32_t device, IcpQueue **out) {
    if (device < 0 || device >= 64) return set_err(nullptr, FS2_ERR_ARG, "bad device %d", device);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev)
        return set_err(nullptr, FS2_ERR_HIP, "no HIP device %d (libfs2 has no CPU path)", device);
    SHIP(hipSetDevice(device));
    IcpQueue &q = g_icpq[device];
    if (!q.stream) {
        SHIP(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking));
        for (IcpSlot &s : q.slot) {
            SHIP(hipHostMalloc((void **)&s.host, 2 * kIcpCloud + 64, hipHostMallocDefault));
            SHIP(hipMalloc(&s.dev, 2 * kIcpCloud + 64));
            SHIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        }
    }
    *out = &q;
    return FS2_OK;
}

}  // namespace

extern "C" {

int fs2_icp_submit(int32_t device, const double *src, int32_t n_src, const double *tgt, int32_t n_tgt,
                   int32_t max_iterations, double threshold, int64_t *ticket) {
    if (n_src <= 0 || n_tgt <= 0 || n_src > 1024 || n_tgt > 1024 || !src || !tgt || !ticket)
        return set_err(nullptr, FS2_ERR_ARG, "fs2_icp_submit: bad arguments (point counts must be 1..1024)");
    std::lock_guard<std::mutex> lk(g_icpq_mu);
    IcpQueue *q = nullptr;
    int rc = icpq_get(device, &q);
    if (rc) return rc;
    IcpSlot &s = q->slot[q->next % kIcpSlots];
    if (s.ticket >= 0)
        return set_err(nullptr, FS2_ERR_STATE, "fs2_icp_submit: %d alignments already outstanding on device %d",
                       kIcpSlots, device);
    // the slot's previous alignment has been waited on, so its buffers are free
    std::memcpy(s.host, src, (size_t)n_src * 16);
    std::memcpy(s.host + kIcpCloud, tgt, (size_t)n_tgt * 16);
    double *ds = (double *)s.dev, *dt = (double *)(s.dev + kIcpCloud);
    double *dR = (double *)(s.dev + 2 * kIcpCloud), *dT = dR + 4;
    int32_t *dI = (int32_t *)(dT + 2);
    SHIP(hipMemcpyAsync(ds, s.host, (size_t)n_src * 16, hipMemcpyHostToDevice, q->stream));
    SHIP(hipMemcpyAsync(dt, s.host + kIcpCloud, (size_t)n_tgt * 16, hipMemcpyHostToDevice, q->stream));
    SHIP(launch_icp(1, n_src, ds, dt, n_tgt, max_iterations, threshold, dR, dT, dI, q->stream));
    SHIP(hipMemcpyAsync(s.host + 2 * kIcpCloud, dR, 52, hipMemcpyDeviceToHost, q->stream));
    SHIP(hipEventRecord(s.done, q->stream));
    s.ticket = q->next++;
    *ticket = s.ticket;
    return FS2_OK;
}

int fs2_icp_wait(int32_t device, int64_t ticket, double R[4], double t[2], int32_t *iterations) {
    if (!R || !t || ticket < 0) return set_err(nullptr, FS2_ERR_ARG, "fs2_icp_wait: bad arguments");
    IcpSlot *s = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_icpq_mu);
        if (device < 0 || device >= 64 || !g_icpq[device].stream)
            return set_err(nullptr, FS2_ERR_STATE, "fs2_icp_wait: nothing submitted on device %d", device);
        s = &g_icpq[device].slot[ticket % kIcpSlots];
        if (s->ticket != ticket)
            return set_err(nullptr, FS2_ERR_STATE, "fs2_icp_wait: ticket %lld is not outstanding",
                           (long long)ticket);
    }
    SHIP(hipEventSynchronize(s->done));
    const double *out = (const double *)(s->host + 2 * kIcpCloud);
    std::memcpy(R, out, 32);
    t[0] = out[4];
    t[1] = out[5];
    if (iterations) std::memcpy(iterations, out + 6, 4);
    std::lock_guard<std::mutex> lk(g_icpq_mu);
    s->ticket = -1;
    return FS2_OK;
}

int fs2_best_fit_transform(int32_t device, const double *src, const double *tgt, int32_t n, double R[4],
                           double t[2]) {
    if (n <= 0 || !src || !tgt || !R || !t) return set_err(nullptr, FS2_ERR_ARG, "fs2_best_fit_transform: bad arguments");
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const size_t b = al16((size_t)n * 16);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, 2 * b + 64, &sc);
    if (rc) return rc;
    double *ds = (double *)sc->buf, *dt = (double *)(sc->buf + b), *dRt = (double *)(sc->buf + 2 * b);
    SHIP(hipMemcpyAsync(ds, src, (size_t)n * 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(hipMemcpyAsync(dt, tgt, (size_t)n * 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(launch_best_fit(ds, dt, n, dRt, sc->stream));
    double out[6];
    SHIP(hipMemcpyAsync(out, dRt, 48, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipStreamSynchronize(sc->stream));
    std::memcpy(R, out, 32);
    t[0] = out[4];
    t[1] = out[5];
    return FS2_OK;
}

int32_t fs2_gaussian_taps(double sigma, double truncate, double *taps, int32_t max_taps) {
    const int32_t r = (int32_t)(truncate * sigma + 0.5);
    if (r < 0 || 2 * r + 1 > max_taps || !taps) return -1;
    const double s2 = sigma * sigma;
    double sum = 0.0;
    std::vector<double> phi(2 * r + 1);
    for (int32_t k = -r; k <= r; ++k) phi[k + r] = std::exp(-0.5 / s2 * (double)(k * k));
    for (double v : phi) sum += v;
    for (int32_t k = 0; k < 2 * r + 1; ++k) taps[k] = phi[2 * r - k] / sum;
    return r;
}

int fs2_line_filter(int32_t device, const double *points, int32_t n, const double *taps, int32_t radius,
                    double *out) {
    if (n < 0 || radius < 0 || (n > 0 && (!points || !out)) || !taps)
        return set_err(nullptr, FS2_ERR_ARG, "fs2_line_filter: bad arguments");
    if (n == 0) return FS2_OK;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const size_t bp = al16((size_t)n * 16), bt = al16((size_t)(2 * radius + 1) * 8);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, 2 * bp + bt, &sc);
    if (rc) return rc;
    double *din = (double *)sc->buf, *dout = (double *)(sc->buf + bp), *dtap = (double *)(sc->buf + 2 * bp);
    SHIP(hipMemcpyAsync(din, points, (size_t)n * 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(hipMemcpyAsync(dtap, taps, (size_t)(2 * radius + 1) * 8, hipMemcpyHostToDevice, sc->stream));
    SHIP(launch_line_filter(din, n, dtap, radius, dout, sc->stream));
    SHIP(hipMemcpyAsync(out, dout, (size_t)n * 16, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipStreamSynchronize(sc->stream));
    return FS2_OK;
}

int fs2_associate(int32_t device, const double observed[2], const double *lm, int32_t L, double gate,
                  int32_t *index) {
    if (!observed || !index || L < 0 || (L > 0 && !lm)) return set_err(nullptr, FS2_ERR_ARG, "fs2_associate: bad arguments");
    if (L == 0) {
        *index = -1;
        return FS2_OK;
    }
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const size_t bl = al16((size_t)L * 48);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, bl + 32, &sc);
    if (rc) return rc;
    double *dl = (double *)sc->buf, *dobs = (double *)(sc->buf + bl);
    int32_t *dout = (int32_t *)(dobs + 2);
    SHIP(hipMemcpyAsync(dl, lm, (size_t)L * 48, hipMemcpyHostToDevice, sc->stream));
    SHIP(hipMemcpyAsync(dobs, observed, 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(launch_associate(dobs, dl, L, gate_to_q(gate), dout, sc->stream));
    int32_t r = -1;
    SHIP(hipMemcpyAsync(&r, dout, 4, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipStreamSynchronize(sc->stream));
    if (r == -2) return set_err(nullptr, FS2_ERR_LINALG, "Singular matrix");
    *index = r;
    return FS2_OK;
}

int fs2_mahalanobis(int32_t device, const double *a, const double *b, const double *cov, int32_t K,
                    double *out) {
    if (K < 0 || (K > 0 && (!a || !b || !cov || !out)))
        return set_err(nullptr, FS2_ERR_ARG, "fs2_mahalanobis: bad arguments");
    if (K == 0) return FS2_OK;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const size_t b2 = al16((size_t)K * 16), b4 = al16((size_t)K * 32), b1 = al16((size_t)K * 8);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, 2 * b2 + b4 + b1 + 16, &sc);
    if (rc) return rc;
    double *da = (double *)sc->buf, *db = (double *)(sc->buf + b2), *dc = (double *)(sc->buf + 2 * b2);
    double *dout = (double *)(sc->buf + 2 * b2 + b4);
    int32_t *dsing = (int32_t *)(sc->buf + 2 * b2 + b4 + b1);
    SHIP(hipMemsetAsync(dsing, 0, 4, sc->stream));
    SHIP(hipMemcpyAsync(da, a, (size_t)K * 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(hipMemcpyAsync(db, b, (size_t)K * 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(hipMemcpyAsync(dc, cov, (size_t)K * 32, hipMemcpyHostToDevice, sc->stream));
    SHIP(launch_mahalanobis(da, db, dc, K, dout, dsing, sc->stream));
    int32_t sing = 0;
    SHIP(hipMemcpyAsync(out, dout, (size_t)K * 8, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipMemcpyAsync(&sing, dsing, 4, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipStreamSynchronize(sc->stream));
    if (sing) return set_err(nullptr, FS2_ERR_LINALG, "Singular matrix");
    return FS2_OK;
}

// ---- numpy's legacy RandomState on the device (fs2_mtrng.hpp / .hip) ----

// A few host threads for fs2_mt_draw's log recomputations (~5 % of 10^6 attempts
// per draw): started on first use, one job at a time, the caller takes a share.
namespace {
struct HostPool {
    std::mutex job_mu, mu;
    std::condition_variable cv, cv_done;
    std::vector<std::thread> th;
    const std::function<void(int64_t, int64_t)> *fn = nullptr;
    int64_t n = 0, chunk = 0;
    std::atomic<int64_t> next{0};
    uint64_t gen = 0;
    int left = 0;
    bool stop = false;
    pid_t owner = getpid();                    // a forked child has none of the threads
    HostPool() {
        cpu_set_t cs;
        int ncpu = 4;
        if (sched_getaffinity(0, sizeof cs, &cs) == 0) ncpu = CPU_COUNT(&cs);
        const int nw = std::max(0, std::min(7, ncpu / 2 - 1));
        for (int i = 0; i < nw; ++i) th.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : th) t.join();
    }
    void work() {
        for (;;) {
            const int64_t k0 = next.fetch_add(chunk);
            if (k0 >= n) return;
            (*fn)(k0, std::min(n, k0 + chunk));
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
            }
            work();
            {
                std::lock_guard<std::mutex> lk(mu);
                if (--left == 0) cv_done.notify_one();
            }
        }
    }
    void run(int64_t count, int64_t ch, const std::function<void(int64_t, int64_t)> &f) {
        std::lock_guard<std::mutex> jl(job_mu);
        {
            std::lock_guard<std::mutex> lk(mu);
            fn = &f;
            n = count;
            chunk = ch;
            next.store(0);
            left = (int)th.size();
            ++gen;
        }
        cv.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu);
        cv_done.wait(lk, [&] { return left == 0; });
    }
};
}  // namespace

// f over [0, count) in chunks of `chunk`, on the pool when it pays
static void host_pool_run(int64_t count, int64_t chunk, const std::function<void(int64_t, int64_t)> &f) {
    if (count <= 2 * chunk) {
        f(0, count);
        return;
    }
    static HostPool pool;
    if (pool.owner != getpid() || pool.th.empty()) {
        f(0, count);
        return;
    }
    pool.run(count, chunk, f);
}

// grow a device / pinned buffer pair to hold n elements of `esz` bytes (contents dropped)
static hipError_t mt_grow(void **dev, void **pin, size_t esz, int64_t *cap, int64_t n) {
    if (n <= *cap) return hipSuccess;
    const int64_t c = std::max<int64_t>(n, *cap + *cap / 2);
    if (dev) {
        hipFree(*dev);
        *dev = nullptr;
        hipError_t e = hipMalloc(dev, esz * (size_t)c);
        if (e != hipSuccess) return e;
    }
    if (pin) {
        if (*pin) hipHostFree(*pin);
        *pin = nullptr;
        hipError_t e = hipHostMalloc(pin, esz * (size_t)c, 0);
        if (e != hipSuccess) return e;
    }
    *cap = c;
    return hipSuccess;
}

// the words R[have, total) of a buffer whose R[0, 624) is a key: in parallel
// regions (jump-ahead) when the buffer is made from its key alone and the draws
// are large, else one workgroup.  Returns the words made (>= total).
static int mt_fill(fs2_handle *h, uint32_t *R, int64_t have, int64_t total, hipStream_t s, int64_t *made) {
    auto &mt = h->mt;
    *made = std::max(have, total);
    if (total <= have) return FS2_OK;
    if (have == kMtN && mt.jG > 1 && total > 3 * mt.jJ) {
        const int64_t par_end = mt.jG * mt.jJ + 1;
        HIP_TRY(h, launch_mt_words_parallel(R, par_end, mt.jpoly, mt_poly_words(), mt.jG, mt.jJ, mt.jwin, s));
        if (total > par_end) HIP_TRY(h, launch_mt_words(R, par_end, total, s));
        *made = std::max(par_end, total);
        return FS2_OK;
    }
    HIP_TRY(h, launch_mt_words(R, have, total, s));
    return FS2_OK;
}

// The device draw is numpy's bit for bit only if the host libm's log is within
// 0.52 ulp (outside the listed midpoint window its result is then forced, and the
// device's double-double log gives it).  Checked once per process on a fixed
// sample: the host restatement of the device log (mt_log) against std::log.
static bool mt_libm_agrees() {
    static const bool ok = [] {
        double thi[kMtLogTab], tlo[kMtLogTab];
        for (int k = 0; k < kMtLogTab; ++k) {
            const DD l = mt_log_tab_entry(k);
            thi[k] = l.hi;
            tlo[k] = l.lo;
        }
        uint64_t z = 0x9E3779B97F4A7C15ull;
        for (int k = 0; k < 8192; ++k) {
            z = z * 6364136223846793005ull + 1442695040888963407ull;
            const double x = (double)((z >> 11) + 1) * 0x1p-53;      // (0, 1], like r2
            bool amb = false;
            const double d = mt_log(x, thi, tlo, &amb);
            if (!amb && d != std::log(x)) return false;
        }
        return true;
    }();
    return ok;
}


// one attempt: the words through the last one it may read, then the draw and
// its counts (to meta_pin, not yet waited for)
static int mt_attempt(fs2_handle *h, MtCtx &c, hipStream_t s) {
    auto &mt = h->mt;
    const int64_t par_words = mt.jG > 1 ? mt.jG * mt.jJ + 1 : 0;   // a parallel fill makes this many
    // words: the key, then through the block holding the u0 words after the last attempt
    const int64_t need = c.pos0 + 4 * c.A + 2;
    c.total = std::max<int64_t>(kMtN, (need + kMtN - 1) / kMtN * kMtN);
    if (c.have == 0) {
        HIP_TRY(h, mt_grow((void **)&mt.raw[mt.cur], nullptr, 4, &mt.raw_cap[mt.cur], std::max(c.total, par_words)));
        std::memcpy(mt.words_pin, c.in.key, sizeof(uint32_t) * kMtN);
        HIP_TRY(h, hipMemcpyAsync(mt.raw[mt.cur], mt.words_pin, sizeof(uint32_t) * kMtN, hipMemcpyHostToDevice, s));
        c.have = kMtN;
    } else if (c.total > mt.raw_cap[mt.cur]) {
        // keep the words made so far
        uint32_t *nr = nullptr;
        const int64_t cap = std::max<int64_t>(c.total, mt.raw_cap[mt.cur] + mt.raw_cap[mt.cur] / 2);
        HIP_TRY(h, hipMalloc((void **)&nr, 4 * (size_t)cap));
        HIP_TRY(h, hipMemcpyAsync(nr, mt.raw[mt.cur], 4 * (size_t)c.have, hipMemcpyDeviceToDevice, s));
        HIP_TRY(h, hipStreamSynchronize(s));
        hipFree(mt.raw[mt.cur]);
        mt.raw[mt.cur] = nr;
        mt.raw_cap[mt.cur] = cap;
    }
    uint32_t *raw = mt.raw[mt.cur];
    const int64_t nb = (c.A + 255) / 256;
    HIP_TRY(h, mt_grow((void **)&mt.boff, nullptr, 4, &mt.boff_cap, std::max<int64_t>(nb, 1)));
    // the listed logs and the results go straight into (mapped) host memory: no
    // result copy after the draw -- a copy is a blit kernel that would queue
    // behind, or slow, the candidate pass beside it
    int64_t acap = mt.amb_cap;
    HIP_TRY(h, mt_grow(nullptr, (void **)&mt.amb_pin, sizeof(MtAmb), &acap, c.amb_cap));
    mt.amb_cap = acap;
    MtAmb *amb_dev = mt.amb_pin;
    MtMeta *meta_host_dev = mt.meta_pin;
    if (hipHostGetDevicePointer((void **)&amb_dev, mt.amb_pin, 0) != hipSuccess) {
        (void)hipGetLastError();
        amb_dev = mt.amb_pin;
    }
    if (hipHostGetDevicePointer((void **)&meta_host_dev, mt.meta_pin, 0) != hipSuccess) {
        (void)hipGetLastError();
        meta_host_dev = mt.meta_pin;
    }
    {
        int64_t made = 0;
        const int rcf = mt_fill(h, raw, c.have, c.total, s, &made);
        if (rcf) return rcf;
        c.have = made;
    }
    HIP_TRY(h, hipMemsetAsync(mt.meta, 0, sizeof(MtMeta), s));
    HIP_TRY(h, launch_mt_draw(raw, c.pos0, (c.pos0 - c.in.pos) / kMtN, c.A, c.P, c.N, c.h0, c.in.gauss, c.sigma, h->first,
                              h->n, h->noise_dev, mt.boff, mt.meta, amb_dev,
                              (int32_t)std::min<int64_t>(mt.amb_cap, INT32_MAX), mt.tab, mt.tab_ready ? 1 : 0,
                              meta_host_dev, s));
    mt.tab_ready = true;
    return FS2_OK;
}

static int mt_begin(fs2_handle *h, const fs2_mt_state *in, double sigma, fs2_mt_state *after, fs2_mt_state *after_u0,
                    double *u0_out, hipStream_t s, MtCtx &c) {
    if (!in || !after || !after_u0) return set_err(&h->err, FS2_ERR_ARG, "fs2_mt_draw: null state");
    if (!(sigma >= 0.0))   // numpy: ValueError for a negative (or NaN) scale
        return set_err(&h->err, FS2_ERR_ARG, "fs2_mt_draw: scale < 0");
    if (in->pos < 0 || in->pos > kMtN || (in->has_gauss != 0 && in->has_gauss != 1))
        return set_err(&h->err, FS2_ERR_ARG, "fs2_mt_draw: bad state (pos %d, has_gauss %d)", in->pos, in->has_gauss);
    if (h->pending.on) return set_err(&h->err, FS2_ERR_STATE, "a submitted scan is pending (fs2_iterate_wait first)");
    if (!mt_libm_agrees())
        return set_err(&h->err, FS2_ERR_STATE,
                       "fs2_mt_draw: this process's libm log is outside the 0.52-ulp bound the device draw relies on "
                       "(draw with numpy on the host)");
    auto &mt = h->mt;
    c = MtCtx{};
    c.in = *in;
    c.sigma = sigma;
    c.after = after;
    c.after_u0 = after_u0;
    c.u0_out = u0_out;
    c.N = h->n_global;
    c.h0 = (c.N > 0 && in->has_gauss) ? 1 : 0;
    c.P = (c.N > c.h0) ? (c.N - c.h0 + 1) / 2 : 0;     // accepted attempts (pairs) needed
    // attempts until P successes at p = pi/4: mean P/p, sd sqrt(P(1-p))/p; 12 sd of margin
    const double mean = (double)c.P / 0.78539816339744831,
                 sd = std::sqrt((double)c.P * 0.21460183660255169) / 0.78539816339744831;
    c.A = c.P ? (int64_t)(mean + 12.0 * sd) + 64 : 0;
    c.amb_cap = c.P / 8 + 4096;
    if (mt.jG == 0) {
        // regions of ~160 K words (16 for 10^6 particles), J >= 2 x 20 561 (the
        // jump's operands come first); the polynomials are made once (~0.3 s)
        const int64_t tn = (2 * kMtN + 4 * (c.A + 2) + 2 + 2 * kMtN + kMtN - 1) / kMtN * kMtN;
        const int G = (int)std::min<int64_t>(kMtMaxGen, tn / 160000);
        mt.jG = 1;
        if (G >= 2) {
            const int64_t J = std::max<int64_t>((tn + G - 1) / G, 2 * 20561 + 2 * kMtN);
            std::vector<uint64_t> gp;
            if (mt_jump_polys((uint64_t)J, G, gp)) {
                HIP_TRY(h, hipMalloc((void **)&mt.jpoly, sizeof(uint64_t) * gp.size()));
                HIP_TRY(h, hipMalloc((void **)&mt.jwin, sizeof(uint32_t) * kMtN * (G - 1)));
                HIP_TRY(h, hipMemcpy(mt.jpoly, gp.data(), sizeof(uint64_t) * gp.size(), hipMemcpyHostToDevice));
                mt.jG = G;
                mt.jJ = J;
            }
        }
    }
    if (!mt.words_pin) HIP_TRY(h, hipHostMalloc((void **)&mt.words_pin, sizeof(uint32_t) * 2 * kMtN, 0));
    if (!mt.meta) {
        HIP_TRY(h, hipMalloc((void **)&mt.tab, sizeof(double) * 2 * kMtLogTab));
        HIP_TRY(h, hipMalloc((void **)&mt.meta, sizeof(MtMeta)));
        HIP_TRY(h, hipHostMalloc((void **)&mt.meta_pin, sizeof(MtMeta), 0));
    }
    if (!mt.side) {
        HIP_TRY(h, hipStreamCreateWithFlags(&mt.side, hipStreamNonBlocking));
        HIP_TRY(h, hipEventCreateWithFlags(&mt.ev_words, hipEventDisableTiming));
        HIP_TRY(h, hipEventCreateWithFlags(&mt.ev_pre, hipEventDisableTiming));
    }
    // the words made ahead serve this draw if it starts where the last one said
    // numpy would be (after its normals, or after its u0 too)
    c.pos0 = in->pos;
    c.have = 0;                                // words of the buffer already made
    if (mt.pre_valid) {
        for (int k = 0; k < 2 && c.have == 0; ++k) {
            if (mt.pre_spos[k] == in->pos && std::memcmp(mt.pre_key[k], in->key, sizeof mt.pre_key[k]) == 0) {
                mt.cur = 1 - mt.cur;
                c.pos0 = mt.pre_pos0[k];
                c.have = mt.pre_total;
            }
        }
    }
    // the side stream's last work (made ahead, or still reading this buffer) first
    if (mt.pre_valid) HIP_TRY(h, hipStreamWaitEvent(s, mt.ev_pre, 0));
    mt.pre_valid = false;
    return mt_attempt(h, c, s);
}

static int mt_end(fs2_handle *h, MtCtx &c, hipStream_t s) {
    auto &mt = h->mt;
    const int64_t N = c.N, P = c.P;
    const int h0 = c.h0;
    MtMeta meta{};
    for (int attempt = 1;; ++attempt) {
        HIP_TRY(h, hipStreamSynchronize(s));
        meta = *mt.meta_pin;
        if (P > 0 && meta.accepted < P) {      // (about 1e-30 per draw) more attempts
            c.A += c.A / 4 + 1024;
        } else if (meta.amb_n > mt.amb_cap) {
            c.amb_cap = (int64_t)meta.amb_n + 1024;
        } else {
            break;
        }
        if (attempt == 6) return set_err(&h->err, FS2_ERR_STATE, "fs2_mt_draw: attempts did not converge");
        const int rca = mt_attempt(h, c, s);
        if (rca) return rca;
    }
    // the listed logs: libm's log on the host (what numpy's legacy_gauss calls)
    const int64_t na = meta.amb_n;
    if (na > 0) {
        HIP_TRY(h, mt_grow((void **)&mt.pidx, (void **)&mt.pidx_pin, 8, &mt.patch_cap, 2 * na));
        HIP_TRY(h, mt_grow((void **)&mt.pval, (void **)&mt.pval_pin, 8, &mt.pval_cap, 2 * na));
        // entry k patches outputs 2k, 2k + 1 (index -1: not this rank's); split over
        // the host pool's threads when there are many
        const int64_t first = h->first, nl = h->n;
        const double sigma = c.sigma;
        double cached = 0.0;
        bool has_cached = false;
        auto fix = [&](int64_t k0, int64_t k1) {
            for (int64_t k = k0; k < k1; ++k) {
                const MtAmb &e = mt.amb_pin[k];
                const double f = mt_polar_f(e.r2, std::log(e.r2));
                const double g0 = f * e.x2, g1 = f * e.x1;
                const int64_t o = h0 + 2 * e.rank;
                const bool in0 = o >= first && o < first + nl;
                mt.pidx_pin[2 * k] = in0 ? o - first : -1;
                mt.pval_pin[2 * k] = 0.0 + sigma * g0;
                const bool in1 = o + 1 < N && o + 1 >= first && o + 1 < first + nl;
                mt.pidx_pin[2 * k + 1] = in1 ? o + 1 - first : -1;
                mt.pval_pin[2 * k + 1] = 0.0 + sigma * g1;
                if (o + 1 >= N) {              // the pair whose second value stays cached (one at most)
                    cached = g1;
                    has_cached = true;
                }
            }
        };
        host_pool_run(na, 2048, fix);
        if (has_cached) meta.gauss = cached;
        const int64_t np = 2 * na;
        HIP_TRY(h, hipMemcpyAsync(mt.pidx, mt.pidx_pin, sizeof(int64_t) * np, hipMemcpyHostToDevice, s));
        HIP_TRY(h, hipMemcpyAsync(mt.pval, mt.pval_pin, sizeof(double) * np, hipMemcpyHostToDevice, s));
        HIP_TRY(h, launch_mt_patch(h->noise_dev, mt.pidx, mt.pval, np, s));
    }
    // the state after the normals, then after the speculative u0 (two more words;
    // k_mt_final left both in meta)
    fs2_mt_state *after = c.after, *after_u0 = c.after_u0;
    std::memcpy(after->key, meta.key_after, sizeof after->key);
    after->pos = meta.pos_after;
    std::memcpy(after_u0->key, meta.key_after_u0, sizeof after_u0->key);
    after_u0->pos = meta.pos_after_u0;
    if (N == 0) {
        after->has_gauss = c.in.has_gauss;
        after->gauss = c.in.gauss;
    } else if (P == 0) {                       // one normal, the cached one
        after->has_gauss = 0;
        after->gauss = 0.0;
    } else {
        after->has_gauss = meta.has_gauss;
        after->gauss = meta.has_gauss ? meta.gauss : 0.0;
    }
    after_u0->has_gauss = after->has_gauss;
    after_u0->gauss = after->gauss;
    {
        // the next draw's words, made on the side stream while the scan runs: the
        // other buffer starts at the key block of `after` (kb1), which also holds or
        // precedes after_u0's (kb2 = kb1 or kb1 + 1)
        const int64_t E = meta.E;
        const int64_t kb1 = (E == c.pos0) ? (c.pos0 - c.in.pos) / kMtN : (E - 1) / kMtN;
        const int64_t kb2 = (E + 1) / kMtN;
        const int nx = 1 - mt.cur;
        const int64_t par_words = mt.jG > 1 ? mt.jG * mt.jJ + 1 : 0;
        // the key block kb1 and what follows it, then the rest from the key
        const bool par = mt.jG > 1;
        const int64_t keep = par ? kMtN : c.have - kMtN * kb1;
        int64_t want = std::max<int64_t>(keep, (2 * kMtN + 4 * (c.A + 2) + 2 + kMtN - 1) / kMtN * kMtN);
        HIP_TRY(h, mt_grow((void **)&mt.raw[nx], nullptr, 4, &mt.raw_cap[nx], std::max(want, par_words)));
        HIP_TRY(h, hipEventRecord(mt.ev_words, s));
        HIP_TRY(h, hipStreamWaitEvent(mt.side, mt.ev_words, 0));
        HIP_TRY(h, hipMemcpyAsync(mt.raw[nx], mt.raw[mt.cur] + kMtN * kb1, 4 * (size_t)keep,
                                  hipMemcpyDeviceToDevice, mt.side));
        {
            int64_t made = 0;
            const int rcf = mt_fill(h, mt.raw[nx], keep, want, mt.side, &made);
            if (rcf) return rcf;
            want = made;
        }
        HIP_TRY(h, hipEventRecord(mt.ev_pre, mt.side));
        std::memcpy(mt.pre_key[0], after->key, sizeof mt.pre_key[0]);
        std::memcpy(mt.pre_key[1], after_u0->key, sizeof mt.pre_key[1]);
        mt.pre_spos[0] = after->pos;
        mt.pre_spos[1] = after_u0->pos;
        mt.pre_pos0[0] = after->pos;
        mt.pre_pos0[1] = kMtN * (kb2 - kb1) + after_u0->pos;
        mt.pre_total = want;
        mt.pre_valid = true;
    }
    // u0 = np.random.uniform(0, 1 / N) = 0 + (1/N - 0) legacy_double (fast_slam_2.py:183)
    const uint32_t wu[2] = {meta.w_u0[0], meta.w_u0[1]};
    const double hi = 1.0 / (double)h->n_global;
    const double u0 = 0.0 + (hi - 0.0) * mt_double(mt_temper(wu[0]), mt_temper(wu[1]));
    *h->u0_pin = u0;
    HIP_TRY(h, hipMemcpyAsync(h->u0_dev, h->u0_pin, 8, hipMemcpyHostToDevice, s));
    if (c.u0_out) *c.u0_out = u0;
    return FS2_OK;
}

// completes a deferred draw: its outputs written, the handle's stream ordered
// after its noise and u0 (armed for the scan unless it failed)
static int mt_finish(fs2_handle *h) {
    auto &mt = h->mt;
    if (!mt.deferred) return FS2_OK;
    mt.deferred = false;
    const int rc = mt_end(h, mt.dc, mt.dstream);
    HIP_TRY(h, hipEventRecord(mt.ev_noise, mt.dstream));
    HIP_TRY(h, hipStreamWaitEvent(h->stream, mt.ev_noise, 0));
    if (rc) return rc;
    mt.armed = true;
    return FS2_OK;
}

int fs2_mt_draw(fs2_handle *h, const fs2_mt_state *in, double sigma, fs2_mt_state *after,
                fs2_mt_state *after_u0, double *u0_out) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    int rc = mt_finish(h);                     // a deferred draw first (its outputs are written)
    if (rc) return rc;
    h->mt.armed = false;
    MtCtx c;
    rc = mt_begin(h, in, sigma, after, after_u0, u0_out, h->stream, c);
    if (rc) return rc;
    rc = mt_end(h, c, h->stream);
    if (rc) return rc;
    h->mt.armed = true;
    return FS2_OK;
}

int fs2_mt_draw_deferred(fs2_handle *h, const fs2_mt_state *in, double sigma, fs2_mt_state *after,
                         fs2_mt_state *after_u0, double *u0_out) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    auto &mt = h->mt;
    int rc = mt_finish(h);
    if (rc) return rc;
    mt.armed = false;
    if (!mt.dstream) {
        HIP_TRY(h, hipStreamCreateWithFlags(&mt.dstream, hipStreamNonBlocking));
        HIP_TRY(h, hipEventCreateWithFlags(&mt.ev_in, hipEventDisableTiming));
        HIP_TRY(h, hipEventCreateWithFlags(&mt.ev_noise, hipEventDisableTiming));
    }
    // after everything enqueued so far (the last scan still reads the noise and u0)
    HIP_TRY(h, hipEventRecord(mt.ev_in, h->stream));
    HIP_TRY(h, hipStreamWaitEvent(mt.dstream, mt.ev_in, 0));
    MtCtx &c = mt.dc;
    rc = mt_begin(h, in, sigma, after, after_u0, u0_out, mt.dstream, c);
    if (rc) return rc;
    mt.deferred = true;
    return FS2_OK;
}

int fs2_debug_mt_jump(const uint32_t key[624], uint64_t J, uint32_t out[624]) {
    if (!key || !out) return set_err(nullptr, FS2_ERR_ARG, "fs2_debug_mt_jump: null argument");
    if (!mt_jump_host(key, J, out)) return set_err(nullptr, FS2_ERR_STATE, "MT19937 characteristic polynomial not found");
    return FS2_OK;
}

int64_t fs2_release_cached_memory(void) { return (int64_t)g_chunks.release(); }

int fs2_debug_vm_fail_after_relocate(int32_t on) {
    g_vm_fail_after_relocate.store(on ? 1 : 0);
    return FS2_OK;
}

int fs2_debug_refuse_peer_maps(fs2_handle *h) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "null handle");
    if (h->refs_shared || h->refs_off)
        return set_err(&h->err, FS2_ERR_STATE, "fs2_debug_refuse_peer_maps: the pools are mapped already");
    h->refuse_maps = true;
    return FS2_OK;
}

int fs2_debug_noise(fs2_handle *h, double *out) {
    if (!h || !out) return set_err(h ? &h->err : nullptr, FS2_ERR_ARG, "fs2_debug_noise: null argument");
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    {
        const int rcm = mt_finish(h);
        if (rcm) return rcm;
    }
    HIP_TRY(h, hipMemcpyAsync(h->noise_pin, h->noise_dev, sizeof(double) * h->n, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    std::memcpy(out, h->noise_pin, sizeof(double) * h->n);
    return FS2_OK;
}

int64_t fs2_debug_check_guards(fs2_handle *h, char *first_bad, int64_t len) {
    if (!h) return set_err(nullptr, FS2_ERR_ARG, "fs2_debug_check_guards: null handle");
    if (first_bad && len > 0) first_bad[0] = 0;
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    std::vector<unsigned char> buf(kGuardBytes);
    int64_t bad = 0;
    for (const auto &g : h->guards) {
        HIP_TRY(h, hipMemcpy(buf.data(), g.at, kGuardBytes, hipMemcpyDeviceToHost));
        int64_t k = 0;
        for (unsigned char c : buf) k += c != (unsigned char)kGuardByte;
        if (k && first_bad && len > 0 && !first_bad[0]) std::snprintf(first_bad, (size_t)len, "%s", g.name);
        bad += k;
    }
    return bad;
}

int fs2_debug_weights(fs2_handle *h, int32_t other, double *out) {
    if (!h || !out) return set_err(h ? &h->err : nullptr, FS2_ERR_ARG, "fs2_debug_weights: null argument");
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    HIP_TRY(h, hipMemcpy(out, h->w[other ? 1 - h->cur : h->cur], sizeof(double) * (size_t)h->n, hipMemcpyDeviceToHost));
    return FS2_OK;
}

int64_t fs2_debug_out_src(fs2_handle *h, int32_t *out, int64_t capacity) {
    if (!h || !out || capacity < h->n)
        return set_err(h ? &h->err : nullptr, FS2_ERR_ARG, "fs2_debug_out_src: null argument or capacity < n");
    HIP_TRY(h, hipSetDevice(h->cfg.device));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    HIP_TRY(h, hipMemcpy(out, h->out_src, sizeof(int32_t) * (size_t)h->n, hipMemcpyDeviceToHost));
    return h->n;
}

int fs2_debug_mt_log(int32_t device, const double *x, int64_t n, double *out, int32_t *amb, int32_t on_host) {
    if (n < 0 || (n > 0 && (!x || !out || !amb))) return set_err(nullptr, FS2_ERR_ARG, "fs2_debug_mt_log: bad arguments");
    if (on_host) {
        double thi[kMtLogTab], tlo[kMtLogTab];
        for (int k = 0; k < kMtLogTab; ++k) {
            const DD l = mt_log_tab_entry(k);
            thi[k] = l.hi;
            tlo[k] = l.lo;
        }
        for (int64_t k = 0; k < n; ++k) {
            bool a = false;
            out[k] = mt_log(x[k], thi, tlo, &a);
            amb[k] = a ? 1 : 0;
        }
        return FS2_OK;
    }
    if (n == 0) return FS2_OK;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const size_t b8 = al16((size_t)n * 8);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, 2 * b8 + al16((size_t)n * 4), &sc);
    if (rc) return rc;
    double *dx = (double *)sc->buf, *dout = (double *)(sc->buf + b8);
    int32_t *damb = (int32_t *)(sc->buf + 2 * b8);
    SHIP(hipMemcpyAsync(dx, x, (size_t)n * 8, hipMemcpyHostToDevice, sc->stream));
    SHIP(launch_mt_debug_log(dx, n, dout, damb, sc->stream));
    SHIP(hipMemcpyAsync(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipMemcpyAsync(amb, damb, (size_t)n * 4, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipStreamSynchronize(sc->stream));
    return FS2_OK;
}

int fs2_debug_philox(int32_t device, int64_t n, const uint32_t *ctr, const uint32_t *key, uint32_t *out) {
    if (n < 0 || (n > 0 && (!ctr || !key || !out))) return set_err(nullptr, FS2_ERR_ARG, "fs2_debug_philox: bad arguments");
    if (n == 0) return FS2_OK;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const size_t bc = al16((size_t)n * 16), bk = al16((size_t)n * 8);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, 2 * bc + bk, &sc);
    if (rc) return rc;
    uint32_t *dc = (uint32_t *)sc->buf, *dk = (uint32_t *)(sc->buf + bc), *dout = (uint32_t *)(sc->buf + bc + bk);
    SHIP(hipMemcpyAsync(dc, ctr, (size_t)n * 16, hipMemcpyHostToDevice, sc->stream));
    SHIP(hipMemcpyAsync(dk, key, (size_t)n * 8, hipMemcpyHostToDevice, sc->stream));
    SHIP(launch_debug_philox(n, dc, dk, dout, sc->stream));
    SHIP(hipMemcpyAsync(out, dout, (size_t)n * 16, hipMemcpyDeviceToHost, sc->stream));
    SHIP(hipStreamSynchronize(sc->stream));
    return FS2_OK;
}

int fs2_debug_normals(int32_t device, uint64_t seed, uint64_t stream, uint64_t first, int64_t n, double *out) {
    if (n < 0 || (n > 0 && !out)) return set_err(nullptr, FS2_ERR_ARG, "fs2_debug_normals: bad arguments");
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    const int64_t chunk = 1 << 24;
    Scratch *sc = nullptr;
    int rc = scratch_get(device, (size_t)std::min(n, chunk) * 8 + 16, &sc);
    if (rc) return rc;
    for (int64_t o = 0; o < n; o += chunk) {
        const int64_t k = std::min(chunk, n - o);
        SHIP(launch_debug_normals(seed, stream, first + (uint64_t)o, k, (double *)sc->buf, sc->stream));
        SHIP(hipMemcpyAsync(out + o, sc->buf, (size_t)k * 8, hipMemcpyDeviceToHost, sc->stream));
        SHIP(hipStreamSynchronize(sc->stream));
    }
    return FS2_OK;
}

#ifdef FS2_PHASE_TIMING
// timing builds only (not in include/fs2.h): summed per-wave s_memtime cycles of
// the k_update phases since the last reset
int fs2_debug_phase_times(uint64_t out[8], int32_t reset) {
    return fs2::debug_phase_times(reinterpret_cast<unsigned long long *>(out), reset) == hipSuccess
               ? FS2_OK
               : FS2_ERR_HIP;
}
extern "C" int fs2_debug_chain_times(uint64_t out[8], int32_t reset) {
    return fs2::debug_chain_times(reinterpret_cast<unsigned long long *>(out), reset) == hipSuccess ? FS2_OK
                                                                                                    : FS2_ERR_HIP;
}
extern "C" int fs2_debug_tail_times(uint64_t out[32], int32_t reset) {
    unsigned long long a[32], b[32], c[32];
    if (fs2::debug_tail_times_update(a, reset) != hipSuccess || fs2::debug_tail_times_exact(b, reset) != hipSuccess ||
        fs2::debug_tail_times_resample(c, reset) != hipSuccess)
        return FS2_ERR_HIP;
    for (int k = 0; k < 32; ++k) out[k] = a[k] + b[k] + c[k];
    return FS2_OK;
}
extern "C" int fs2_debug_finalize_times(uint64_t out[8], int32_t reset) {
    return fs2::debug_fin_times(reinterpret_cast<unsigned long long *>(out), reset) == hipSuccess ? FS2_OK
                                                                                                  : FS2_ERR_HIP;
}
extern "C" int fs2_debug_icp_phase_times(uint64_t out[4], int32_t reset) {
    return fs2::debug_icp_phase_times(reinterpret_cast<unsigned long long *>(out), reset) == hipSuccess
               ? FS2_OK
               : FS2_ERR_HIP;
}
#endif

int fs2_cluster_points(int32_t device, const double *points, int64_t n, double eps, int64_t min_samples,
                       double *centres, int64_t cap, int64_t *n_clusters, int32_t *labels, int32_t where) {
    if (n <= 0 || !points || !n_clusters || !(eps > 0.0) || min_samples < 1 || cap < 0 || (cap > 0 && !centres))
        return set_err(nullptr, FS2_ERR_ARG, "fs2_cluster_points: bad arguments (n > 0, eps > 0, min_samples >= 1)");
    if (n > (int64_t)INT32_MAX) return set_err(nullptr, FS2_ERR_ARG, "fs2_cluster_points: more than 2^31 points");
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, 16, &sc);
    if (rc) return rc;
    const double2 *dp = reinterpret_cast<const double2 *>(points);
    double2 *own = nullptr;
    if (where != FS2_DEVICE) {
        SHIP(hipMalloc(&own, sizeof(double2) * n));
        SHIP(hipMemcpyAsync(own, points, sizeof(double2) * n, hipMemcpyHostToDevice, sc->stream));
        dp = own;
    }
    int32_t status = 0;
    int64_t K = 0;
    hipError_t e = cluster_points(dp, n, eps, min_samples, cap > 0 ? centres : nullptr, cap, &K, labels, &status,
                                  sc->stream);
    if (own) (void)hipFree(own);
    if (e != hipSuccess) return set_err(nullptr, FS2_ERR_HIP, "fs2_cluster_points: %s", hipGetErrorString(e));
    if (status == 1) return set_err(nullptr, FS2_ERR_ARG, "Input contains NaN or infinity");
    if (status == 2) return set_err(nullptr, FS2_ERR_ARG, "point coordinates span too many eps-cells");
    *n_clusters = K;
    if (K > cap) return set_err(nullptr, FS2_ERR_ARG, "%lld clusters, centre buffer holds %lld", (long long)K,
                                (long long)cap);
    return FS2_OK;
}

// fs2_frontend: the batched device pipeline (fs2_frontend.hip) up to the corners;
// the corners' (distance, angle) (GeometryUtils.calculate_distance_and_angle,
// geometry_utils.py:65-74: math.sqrt(x ** 2 + y ** 2), math.atan2(y, x)) on the
// host with the C library's powf / pow / atan2 -- the functions numpy's scalar
// power and math.atan2 call -- so the measurements fed to fs2_iterate are the
// reference's bits.  Called through volatile pointers so that the compiler
// cannot rewrite pow(x, 2) as x * x (which differs in the last bit at times).
static float (*volatile g_powf)(float, float) = powf;
static double (*volatile g_pow)(double, double) = pow;

int fs2_frontend(int32_t device, int32_t B, const int64_t *offsets, const double *points, int32_t where,
                 const double *taps, int32_t radius, int32_t legacy, fs2_frontend_out *out) {
    if (B < 0 || !offsets || !taps || radius < 0 || !out || !out->counts || out->cap < 0 ||
        (legacy != 0 && legacy != 1))
        return set_err(nullptr, FS2_ERR_ARG, "fs2_frontend: bad arguments");
    if (B == 0) return FS2_OK;
    if (offsets[0] != 0) return set_err(nullptr, FS2_ERR_ARG, "fs2_frontend: offsets[0] must be 0");
    for (int32_t b = 0; b < B; ++b)
        if (offsets[b + 1] < offsets[b]) return set_err(nullptr, FS2_ERR_ARG, "fs2_frontend: offsets decrease");
    if (offsets[B] > 0 && !points) return set_err(nullptr, FS2_ERR_ARG, "fs2_frontend: null points");
    if (offsets[B] >= ((int64_t)1 << 31) / 13)
        return set_err(nullptr, FS2_ERR_ARG, "fs2_frontend: too many points in one call");
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    Scratch *sc = nullptr;
    int rc = scratch_get(device, 16, &sc);
    if (rc) return rc;
    static FeWorkspace ws[64];
    FeArgs a;
    a.B = B;
    a.offs = offsets;
    a.points = points;
    a.points_on_device = where == FS2_DEVICE;
    a.taps = taps;
    a.radius = radius;
    a.legacy = legacy;
    a.cap = out->cap;
    FeHostOut o;
    o.lines = out->lines;
    o.intersections = out->intersections;
    o.clusters = out->clusters;
    std::vector<double> corners;
    const bool want_corners = out->corners || out->measurements;
    if (want_corners) {
        corners.resize((size_t)B * std::max(out->cap, 1) * 2);
        o.corners = corners.data();
    }
    hipError_t e = frontend_run(ws[device], a, o, sc->stream);
    if (e != hipSuccess) return set_err(nullptr, FS2_ERR_HIP, "fs2_frontend: %s", hipGetErrorString(e));
    for (int32_t b = 0; b < B; ++b) {
        switch (o.status[b]) {
        case kFeOk: break;
        case kFeEmpty: return set_err(nullptr, FS2_ERR_ARG, "scan %d has no points (zero-size array)", b);
        case kFeNonFinite: return set_err(nullptr, FS2_ERR_ARG, "scan %d has non-finite points", b);
        case kFeTooLarge:
            return set_err(nullptr, FS2_ERR_ARG, "scan %d spans more than %d px of Hough image", b, kFeMaxRow / 2 - 1);
        default: return set_err(nullptr, FS2_ERR_ARG, "scan %d has more than %d Hough lines", b, kFeMaxLines);
        }
    }
    std::memcpy(out->counts, o.counts.data(), sizeof(int32_t) * 4 * B);
    const int cap = out->cap;
    for (int32_t b = 0; b < B; ++b) {
        const int32_t *c = out->counts + 4 * b;
        if ((out->lines && c[0] > cap) || (out->intersections && c[1] > cap) || (out->clusters && c[2] > cap) ||
            (want_corners && c[3] > cap))
            return set_err(nullptr, FS2_ERR_ARG, "scan %d: counts (%d, %d, %d, %d) exceed cap %d", b, c[0], c[1], c[2],
                           c[3], cap);
    }
    if (want_corners) {
        for (int32_t b = 0; b < B; ++b) {
            const int32_t m = out->counts[4 * b + 3];
            for (int32_t k = 0; k < m; ++k) {
                const size_t r = ((size_t)b * cap + k) * 2;
                const double x = corners[r], y = corners[r + 1];
                if (out->corners) {
                    out->corners[r] = x;
                    out->corners[r + 1] = y;
                }
                if (out->measurements) {
                    double d;
                    if (legacy) {
                        d = std::sqrt(g_pow(x, 2.0) + g_pow(y, 2.0));
                    } else {
                        const float s = g_powf((float)x, 2.0f) + g_powf((float)y, 2.0f);
                        d = std::sqrt((double)s);
                    }
                    out->measurements[r] = d;
                    out->measurements[r + 1] = std::atan2(y, x);
                }
            }
        }
    }
    return FS2_OK;
}

int fs2_comm_unique_id(uint8_t out[128]) {
    if (!out) return set_err(nullptr, FS2_ERR_ARG, "null argument");
    std::string err;
    int rc = fs2comm::unique_id(out, &err);
    if (rc) return set_err(nullptr, rc, "%s", err.c_str());
    return FS2_OK;
}

int fs2_plan_ranges(const double *c, int64_t n, int64_t first_global, int64_t N, double offset, double u0,
                    int32_t *mlo, int32_t *mhi) {
    if ((n > 0 && (!c || !mlo || !mhi)) || n < 0 || first_global < 0 || first_global + n > N || N > INT32_MAX)
        return set_err(nullptr, FS2_ERR_ARG, "fs2_plan_ranges: bad arguments");
    // k_ranges without the exact chain: the running value through particle i
    const bool r0 = first_global == 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t g = first_global + i;
        const double cur = r0 ? c[i] : offset + c[i];
        const double prev = (g == 0) ? 0.0 : ((i == 0) ? offset : (r0 ? c[i - 1] : offset + c[i - 1]));
        int64_t lo, hi;
        plan_range(g, N, prev, cur, u0, lo, hi);
        mlo[i] = (int32_t)lo;
        mhi[i] = (int32_t)hi;
    }
    return FS2_OK;
}

int fs2_plan_sends(const int32_t *mlo, const int32_t *mhi, const int32_t *cnt, int64_t n, int64_t N,
                   int32_t world, int32_t rank, int64_t *run, int64_t *K, int64_t *S) {
    if ((n > 0 && (!mlo || !mhi || !cnt)) || !run || !K || !S || world < 1 || world > kMaxRanks || rank < 0 ||
        rank >= world || n < 0)
        return set_err(nullptr, FS2_ERR_ARG, "fs2_plan_sends: bad arguments");
    // k_pack_plan / k_pack_bounds: exclusive counts of non-empty ranges and their slots
    std::vector<int64_t> E(n + 1, 0), C(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        const bool ne = mlo[i] <= mhi[i];
        E[i + 1] = E[i] + (ne ? 1 : 0);
        C[i + 1] = C[i] + (ne ? cnt[i] : 0);
    }
    for (int p = 0; p < world; ++p) {
        int64_t i0 = 0, i1 = 0;
        if (p != rank)
            plan_run(n, shard_begin(N, world, p), shard_begin(N, world, p + 1), [&](int64_t i) { return (int64_t)mlo[i]; },
                     [&](int64_t i) { return (int64_t)mhi[i]; }, i0, i1);
        run[2 * p] = i0;
        run[2 * p + 1] = i1;
        K[p] = E[i1] - E[i0];
        S[p] = C[i1] - C[i0];
    }
    return FS2_OK;
}

}  // extern "C"
