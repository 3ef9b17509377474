// fs2_kernels.hpp -- kernel parameter blocks and launch wrappers shared by
// fs2_kernels.hip (device code) and fs2_api.hip (host C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fs2 {

constexpr int kBlock = 256;          // 4 waves of 64
constexpr int kPageSlots = 64;       // landmark slots per page
constexpr int kMaxPages = 64;        // 4096 slots per particle max
constexpr int kMaxM = 4;             // measurements fused into one map pass
constexpr int kGroup = 4;            // slots whose mirrors a lane loads per step (64 B)

// A page holds 64 slots of ONE particle's map, contiguous:
//   [0, 1024)     64 x float4 gate mirror (x, y, s, 0)     -- read every scan
//   [1024, 4096)  64 x 48 B fp64 slot (x, y, P00, P01, P10, P11) -- read on candidates
// Arena k holds page k (slots 64k .. 64k+63) of every physical map.
constexpr int kPageBytes = 4096;
constexpr int kMirrorBytes = 1024;
constexpr int kSlotBytes = 48;

// Device statistics of one scan (zeroed before every scan).
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
    int32_t n_copies;        // maps copied by the resample (duplicated particles)
    unsigned long long visited, candidates, hits, appends, written, ambiguous, resample_slots;
};

struct MeasPack {
    double d[kMaxM], b[kMaxM], ox[kMaxM], oy[kMaxM];
    float fx[kMaxM], fy[kMaxM];   // fp32 observed point for the gate mirror
    float fe[kMaxM];              // >= |ox - fx|, |oy - fy| (rounded up)
};

// Logical particle m's map lives in physical map phys[m]; resampling
// re-points phys instead of moving most maps.
struct MapRef {
    char *const *arenas;     // device array: arena k = page k of every physical map
    const int32_t *phys;     // logical -> physical map
};

struct UpdateParams {
    int64_t n;               // local particles
    int64_t gidx0;           // global index of local particle 0
    double *x, *y, *yaw, *w;
    int32_t *cnt;
    MapRef map;
    const double *noise;     // injected normal draws (nullable -> Philox)
    uint64_t seed, scan;
    double sigma;            // std of the selected motion noise
    double rotation, translation;
    int32_t do_move;
    int32_t m;               // measurements in this pass
    int32_t k0;              // first measurement index of this pass
    int32_t last_pass;
    double gate2;            // match iff 0 <= q < gate2  (sqrt(q) < gate)
    float gate2f;            // gate2 rounded up to fp32 (mirror test)
    int32_t filter;          // use the fp32 gate mirror
    double R[4];
    double init_cov[4];
    int32_t *assoc;          // [M][n] or null
    double *wpart;           // [gridDim.x] block partial sums of w (last pass)
    DevStats *stats;
    MeasPack meas;
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
    double *part_sq;         // normalise partials: sum w'^2
    double *part_best_w;
    int64_t *part_best_i;
    int32_t *part_maxcnt;
    int32_t nparts;
    double floor;
    int32_t sequential;
    const double *u0_host;   // nullable: injected u0 value lives here (device copy)
    uint64_t seed, scan;
    DevStats *stats;
};

struct ResampleParams {
    int64_t n;
    double *w;               // normalised weights (current)
    double *c;               // prefix workspace [n]
    double *bsum;            // block sums (prefix)
    int32_t nblk;            // prefix blocks
    int32_t *src;            // [n] source of each output
    const double *x, *y, *yaw;
    const int32_t *cnt;
    double *ox, *oy, *oyaw, *ow;
    int32_t *ocnt;
    char *const *arenas;
    const int32_t *phys;     // current logical -> physical
    int32_t *ophys;          // next logical -> physical
    int32_t *used;           // [n] particle is a source
    int32_t *rank_d;         // [n] rank among dropped particles
    int32_t *rank_e;         // [n] rank among extra outputs
    int32_t *iblk;           // [2 * nb] per-block counts -> offsets
    int32_t *freelist;       // [n] physical maps of dropped particles
    int32_t *tasks;          // [n] extra outputs to copy
    double *part_best_w;
    int64_t *part_best_i;
    DevStats *stats;
};

// ---- launch wrappers (defined in fs2_kernels.hip) ----
hipError_t launch_update(const UpdateParams &p, hipStream_t s);
hipError_t launch_wsum(const ReduceParams &p, hipStream_t s);
hipError_t launch_normalize(const ReduceParams &p, hipStream_t s);
hipError_t launch_finalize(const ReduceParams &p, hipStream_t s);
hipError_t launch_resample(const ResampleParams &p, int sequential, hipStream_t s);

hipError_t launch_import(const double *stage, const int32_t *cnt_stage, int64_t first,
                         int64_t count, int32_t lm_cap, MapRef map, int32_t *cnt,
                         hipStream_t s);
hipError_t launch_export(double *stage, int64_t first, int64_t count, int32_t lm_cap,
                         MapRef map, const int32_t *cnt, hipStream_t s);
hipError_t launch_fill(double *p, double v, int64_t n, hipStream_t s);
hipError_t launch_iota(int32_t *p, int64_t n, hipStream_t s);

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
