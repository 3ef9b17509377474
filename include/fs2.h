/*
 * fs2.h -- C ABI of libfs2.so, the MI355X (gfx950) FastSLAM 2.0 particle-update engine.
 *
 * Drop-in boundary for the reference's `fast_slam_2` hot path (cy-rae/fast-slam).
 * The reference has no FFI of its own: it is pure Python, and its callers use the
 * object API `FastSLAM2().iterate(rotation, translation, measurements)` plus the
 * static helpers of ICP / LineFilter / LandmarkUtils / GeometryUtils.  Each entry
 * point below names the reference interface it replaces (file:line under
 * /root/reference).  The Python shim fast-slam_amd/fast_slam_2/ binds these with
 * ctypes.
 *
 * Conventions:
 *   - plain C types only; every entry point returns FS2_OK (0) or a negative
 *     FS2_ERR_* code; fs2_last_error() gives the message;
 *   - the caller owns every array it passes; the library copies in/out and never
 *     keeps caller pointers;
 *   - a handle is bound to one HIP device and one stream (and, with
 *     world_size > 1, one RCCL rank); it is not thread-safe;
 *   - all state is fp64 like the reference.
 */
#ifndef FS2_H
#define FS2_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FS2_ABI_VERSION 2

enum {
    FS2_OK = 0,
    FS2_ERR_ARG = -1,       /* invalid argument */
    FS2_ERR_HIP = -2,       /* HIP runtime error (no device, launch failure, ...) */
    FS2_ERR_OOM = -3,       /* device allocation failed */
    FS2_ERR_LINALG = -4,    /* singular covariance: reference raises numpy.linalg.LinAlgError */
    FS2_ERR_STATE = -5,     /* call not valid in the current state */
    FS2_ERR_COMM = -6,      /* RCCL error */
    FS2_ERR_CAPACITY = -7   /* a map needs more landmark slots than allowed */
};

/* Reduction order for normalise / N_eff / resample prefix.  The reference sums
 * the weights with Python's sum (fast_slam_2.py:166), the resample's running
 * sum one particle at a time (:184-193) and sum(w^2) with numpy (:219-223). */
enum {
    FS2_REDUCE_AUTO = 0,       /* one GPU: SEQUENTIAL up to 4096 particles, EXACT above;
                                  sharded: EXACT when every shard holds >= 8192 particles
                                  (and <= 8M), else PARALLEL */
    FS2_REDUCE_SEQUENTIAL = 1, /* the reference's summation orders, one lane */
    FS2_REDUCE_PARALLEL = 2,   /* fixed-order trees (deterministic, not the reference's
                                  rounding); fs2_iter_stats.reduce_ambiguous counts the
                                  decisions that rounding could flip */
    FS2_REDUCE_EXACT = 3       /* the reference's summation orders, bit-exact, evaluated by
                                  parallel kernels; sharded: across the ranks in the global
                                  particle order (FS2_ERR_ARG at creation where shards are
                                  too small: fewer than 8192 particles) */
};

enum { FS2_HOST = 0, FS2_DEVICE = 1 };   /* where caller buffers live */

/* How sharded ranks (world_size > 1) talk. */
enum {
    FS2_COMM_RCCL = 0,      /* one process per GPU, RCCL over xGMI; comm_id from fs2_comm_unique_id */
    FS2_COMM_LOCAL = 1,     /* ranks are threads of one process (testing); comm_id is a group key */
    FS2_COMM_SHM = 2        /* ranks are processes on one host (any GPUs, several may share one):
                               stream-ordered collectives through a POSIX shared-memory segment
                               named from comm_id (a random group key, e.g. 128 urandom bytes) */
};

typedef struct fs2_handle fs2_handle;

typedef struct fs2_config {
    int64_t num_particles;          /* NUM_PARTICLES, global over all ranks (config.py:7) */
    double translation_noise;       /* TRANSLATION_NOISE (config.py:11) */
    double rotation_noise;          /* ROTATION_NOISE (config.py:12) */
    double measurement_noise[4];    /* MEASUREMENT_NOISE, row-major 2x2 (config.py:15) */
    double max_landmark_distance;   /* MAXIMUM_LANDMARK_DISTANCE (config.py:18) */
    double init_landmark_cov[4];    /* Landmark default covariance 0.1*I (models/landmark.py:13) */
    double weight_floor;            /* 1e-5 normalise floor (algorithms/fast_slam_2.py:168,173) */
    int32_t landmark_capacity;      /* initial map slots per particle; grows on demand */
    int32_t max_landmark_capacity;  /* hard limit on slots (0 = 4096) */
    int32_t device;                 /* HIP device ordinal */
    int32_t reduce_mode;            /* FS2_REDUCE_* */
    uint64_t seed;                  /* Philox seed for device-drawn noise and u0 */
    int32_t record_assoc;           /* keep per-(measurement, particle) association indices */
    int32_t gate_filter;            /* fp32 conservative gate pre-filter (exactness preserved) */
    int32_t rank;                   /* this rank (particle shard) */
    int32_t world_size;             /* number of ranks; 1 = single GPU */
    uint8_t comm_id[128];           /* ncclUniqueId from fs2_comm_unique_id (world_size > 1) */
    int32_t comm_mode;              /* FS2_COMM_* */
    int32_t sharded_path;           /* 1: run the sharded path (transport, collectives) even
                                       with world_size 1 -- tests the transport on one GPU */
    int64_t page_pool;              /* initial page pool (128-byte pages); 0 = twice the initial
                                       maps plus 8 per particle.  Pools are collected when a
                                       reservation does not fit and grow when a collection
                                       frees too little */
    int64_t record_pool;            /* initial slot-record pool (48 B each); 0 = 1.25x the
                                       initial capacity plus 64 per particle */
    int32_t page_refs;              /* sharded resample: 0 = auto (off: measured slower than sending
                                       pages, and the IPC mapping hung between processes on one GPU,
                                       DESIGN.md §5), 1 = on (2..15 ranks; if a rank cannot map its
                                       peers' pools every rank falls back to pages), -1 = off.
                                       On: a particle that changes ranks travels as its
                                       page-table row of references to pages on the rank that
                                       holds them (every rank maps the others' pools, IPC); the
                                       receiver copies a page when the update pass first needs
                                       it.  Off: each destination gets each distinct page's
                                       content */
    int32_t reserved0;
} fs2_config;

typedef struct fs2_iter_stats {
    int32_t resampled;          /* the N_eff < N/2 rule fired (fast_slam_2.py:62) */
    int32_t max_count;          /* largest map size after the scan */
    double n_eff;               /* __calculate_effective_particles (fast_slam_2.py:212-223) */
    double total_weight;        /* __normalize_weights total (fast_slam_2.py:166) */
    int64_t best_index;         /* global index of the estimate particle */
    uint64_t slots_visited;     /* landmark slots read by the association pass */
    uint64_t candidates;        /* slots whose fp64 data was read (== visited without gate_filter) */
    uint64_t hits;              /* measurement updates that associated (EKF) */
    uint64_t appends;           /* measurement updates that appended a landmark */
    uint64_t slots_written;     /* landmark slots written (EKF updates + appends) */
    uint64_t ambiguous;         /* gate decisions within 1e-9 relative of the threshold */
    uint64_t resample_slots;    /* landmark slots the resampled maps refer to (shared, not copied) */
    int32_t error_flags;        /* bit 0: singular covariance met; bit 1: non-finite weight;
                                   bit 2: a sharded exact-order reduction could not be completed
                                   (a shard's chain ops overflowed, or numpy's chunk edges did not
                                   fit) and the tree estimate stood in -- with reduce_mode EXACT
                                   fs2_iterate_wait then fails with FS2_ERR_STATE, with AUTO the
                                   scan completes and reduce_ambiguous counts it; bit 3: page_refs
                                   localisation ran out of pool room (the scan fails) */
    int32_t reduce_ambiguous;   /* FS2_REDUCE_PARALLEL: resample boundaries (and the N_eff
                                   rule) within the rounding bound of the reference's
                                   summation order, i.e. decisions that may differ from it;
                                   always 0 in the SEQUENTIAL / EXACT modes */
    uint64_t cow_pages;         /* shared 8-slot pages copied before their first write */
    uint64_t new_pages;         /* fresh pages (appends, maps received from other ranks) */
    uint64_t collections;       /* page-pool collections so far (handle lifetime) */
    uint64_t pool_pages;        /* pages in the pool (128 B each) */
    uint64_t pages_opened;      /* pages whose 8 gate mirrors the candidate stream loaded
                                   (the rest were rejected from their descriptor) */
    uint64_t reference_visits;  /* landmarks the reference's first-match scan would read:
                                   j + 1 for a match at j, the map size for an append
                                   (landmark_utils.py:103-117; SURVEY §8d's V) */
    uint64_t pool_records;      /* records in the record pool (48 B each) */
    uint64_t pool_copies;       /* pool growths that moved a pool (allocate and copy) instead of
                                   mapping memory at the end of its reserved range (handle lifetime) */
} fs2_iter_stats;

typedef struct fs2_profile {
    int64_t scans;              /* scans timed since profiling was enabled */
    int64_t update_launches;    /* update passes (candidate stream + exact kernel) */
    double update_ms;           /* summed device time of the update passes (HIP events) */
    double reduce_ms;           /* after the update pass: normalise / N_eff / estimate,
                                   the resample when it fires, stats publication */
    double resample_ms;         /* unused (0): folded into reduce_ms */
    double scan_ms;             /* summed device time of whole scans */
    uint64_t update_bytes;      /* algorithmic bytes moved by the update kernel */
    uint64_t resample_bytes;    /* algorithmic bytes moved by resample gathers */
    int64_t filter_launches;    /* timed candidate-stream launches (k_candidates) */
    double filter_ms;           /* their summed device time (HIP events) */
    uint64_t filter_bytes;      /* their algorithmic bytes (mirrors, lists, counts) */
    int64_t exact_launches;     /* timed exact-association launches (k_update; scans of one pass) */
    double exact_ms;            /* their summed device time (HIP events) */
    int64_t comm_calls;         /* sharded: transport calls and mid-scan waits timed */
    double comm_ms;             /* their summed host wall time (a mid-scan wait includes the
                                   collectives queued before it on the stream) */
    int64_t migrations;         /* sharded: resamples whose plan sent particles to other ranks */
    uint64_t sent_particles;    /* particles sent (one per source and destination) */
    uint64_t sent_rows;         /* their page-table rows */
    uint64_t sent_pages;        /* distinct pages those rows name (sent once per destination) */
    uint64_t sent_bytes;        /* transfer bytes (headers, row entries, pages with their records) */
    double migrate_ms;          /* host wall time from the plan to the end of the exchange */
    uint64_t sent_pages_repeat; /* of sent_pages, those that had gone to the same rank before since
                                   the sender's last collection (what a receiver-side page cache
                                   could skip; a probe, nothing is skipped) */
    /* The counters of the algorithmic byte model, summed over the
     * timed candidate / exact launches, so that filter_bytes and update_bytes can be
     * recomputed from them:
     *   k_candidates: 4 B per streamed descriptor + 128 B per opened page + 8 B per
     *                 list entry + 8 B per particle and pass + 4 B per row box read;
     *   k_update:     model_fixed_bytes (particle scalars, free-list ids, counts)
     *                 + 8 B per list entry + 48 B per candidate record + 68 B per
     *                 written slot (record 48, mirror 16, descriptor read 4)
     *                 + 260 B per copied page (its descriptor written) + 8 B per row
     *                 box read and written. */
    uint64_t model_groups;      /* descriptors streamed */
    uint64_t model_opened;      /* pages whose 128-byte mirror line was loaded */
    uint64_t model_words;       /* candidate list entries */
    uint64_t model_candidates;  /* fp64 records read by the exact pass */
    uint64_t model_written;     /* slots written (modified + appended) */
    uint64_t model_cow;         /* pages copied before their first write */
    uint64_t model_fixed_bytes; /* k_update's per-particle bytes (scalars, ids, counts) */
    uint64_t model_box_bytes;   /* row-box bytes (k_candidates reads, k_update reads + writes) */
    uint64_t localized_pages;   /* page_refs: remote pages copied into this rank's pools before an
                                   update pass read them (with their records: 128 + 8 x 48 B each) */
    int64_t page_refs;          /* page_refs mode: 1 in effect, 0 off, -1 turned off on every rank at
                                   the first scan because some rank could not map its peers' pools
                                   (no peer access between the devices; resamples then send pages) */
    int64_t pool_collections;   /* pool collections run (host calls; each drains the stream) */
    double collect_ms;          /* their host wall time */
    int64_t pool_grows;         /* pool growths (in place, or allocate and copy: fs2_iter_stats.pool_copies) */
    double grow_ms;             /* their host wall time */
    int64_t scan_allocs;        /* buffers reallocated inside a scan's sharded resample (transfer
                                   arenas, dedup table, received rows / pages, page-table rows for a
                                   received map longer than every local one): each drains the stream
                                   and allocates.  Counted whether or not profiling is on; 0 when the
                                   creation-time sizes hold */
    uint64_t recv_bytes;        /* sharded: transfer bytes this rank received at resamples (what must
                                   arrive before its next update pass can run) */
    double exchange_ms;         /* sharded: device time of the resamples' exchanges (HIP events around
                                   the transport's grouped send / receive on the scan's stream; nothing
                                   overlaps them: the exposed exchange time) */
} fs2_profile;

/* ---------------------------------------------------------------- core ---- */

int32_t fs2_abi_version(void);

/* Hash of the sources and flags this library was built from (fast-slam_amd/build.py
 * source_id): the tests refuse a library whose id is not that of the tree they run in. */
const char *fs2_build_id(void);

/* Fills cfg with the reference's config.py defaults (NUM_PARTICLES=20, ...). */
void fs2_config_default(fs2_config *cfg);

/* Replaces FastSLAM2.__init__ (algorithms/fast_slam_2.py:20-31) and
 * Particle.__init__ (models/particle.py:11-20): N particles at (0, 0, 0), weight
 * 1/N, empty maps.  Owns all device memory. */
int fs2_create(const fs2_config *cfg, fs2_handle **out);
void fs2_destroy(fs2_handle *h);

/* Device memory of closed handles kept for reuse: fs2_destroy keeps the physical
 * chunks of the pools that grow in place (up to FS2_VMM_CACHE_MB MiB, read at every close;
 * default 0: nothing is kept, opt in when closing and re-creating large handles) and later handles of the process grow into them before they ask
 * the driver for new memory -- a large allocation right after tens of GB were
 * released waited seconds for the driver.  This releases every
 * kept chunk; returns the bytes released. */
int64_t fs2_release_cached_memory(void);

/* Message for the last error on this handle (h may be NULL: last global error). */
const char *fs2_last_error(const fs2_handle *h);

/* Replaces FastSLAM2.iterate (algorithms/fast_slam_2.py:33-67):
 *   move every particle (:69-87), update with each measurement in order (:90-159),
 *   normalise (:161-175), N_eff (:212-223), low-variance resample when
 *   N_eff < N/2 (:62, :177-199), return the first max-weight pose (:201-210).
 * meas:     M x 2 host array (distance, yaw) -- Measurement.as_vector (models/measurement.py:18-23)
 * observed: M x 2 host array of the robot-frame points d*cos(yaw), d*sin(yaw)
 *           (fast_slam_2.py:100-103) as the caller computed them, or NULL to
 *           compute them here with libm.
 * noise:    NULL -> Philox draws on device; else N_local host values, the
 *           np.random.normal(0, sigma) draw for each particle (fast_slam_2.py:79,81).
 * u0:       NULL -> Philox draw on device; else the np.random.uniform(0, 1/N)
 *           starting point (fast_slam_2.py:183), used only if resampling fires.
 * out_pose: x, y, yaw of the estimate.  stats: nullable. */
int fs2_iterate(fs2_handle *h, double rotation, double translation, const double *meas,
                const double *observed, int32_t M, const double *noise, const double *u0,
                double out_pose[3], fs2_iter_stats *stats);

/* fs2_iterate in two halves: fs2_iterate_submit enqueues the scan (same
 * arguments; on a sharded handle it also performs the mid-scan exchanges) and
 * returns while the GPU works; fs2_iterate_wait completes the oldest submitted
 * scan (pose, stats).  The caller can do host work in between -- e.g. hand the
 * next scan's ICP alignment to the GPU (config 4) -- without delaying the scan.
 *
 * Up to two scans may be outstanding: submit(s + 1), then wait (returns s), then
 * submit(s + 2), wait (returns s + 1), ...  The second submit completes the
 * outstanding scan first and keeps its results for the next wait, so results are
 * identical to one scan at a time and come back in submission order.  A third
 * submit, fs2_iterate, and reading / writing the state (or the associations)
 * while scans are outstanding fail with FS2_ERR_STATE. */
int fs2_iterate_submit(fs2_handle *h, double rotation, double translation, const double *meas,
                       const double *observed, int32_t M, const double *noise, const double *u0);
int fs2_iterate_wait(fs2_handle *h, double out_pose[3], fs2_iter_stats *stats);

/* numpy's legacy global RandomState on the device, for the drop-in iterate()
 * (replaces the host draws np.random.normal(0, ROTATION_NOISE / TRANSLATION_NOISE)
 * of fast_slam_2.py:79,81 for every particle in order, and the resample start
 * np.random.uniform(0, 1 / NUM_PARTICLES) of fast_slam_2.py:183).  The state is
 * np.random.get_state()'s ('MT19937', key, pos, has_gauss, cached_gaussian).
 * fs2_mt_draw draws the N_global normals legacy_normal(0, sigma) from *in -- this
 * rank's slice into the handle's noise buffer -- and the speculative u0 after
 * them; the next fs2_iterate / fs2_iterate_submit (noise and u0 NULL) uses both.
 * *after is numpy's state after the normals, *after_u0 after the u0 draw too
 * (the caller keeps it only if the scan resampled, as the reference draws u0 only
 * then).  Bit for bit with numpy: the MT19937 words, legacy_double, the polar
 * method's rejections and roundings; log(r2) in double-double on the device, the
 * few results within 0.025 ulp of a rounding midpoint recomputed with the host's
 * libm log (glibc's log is within 0.52 ulp, not always correctly rounded). */
typedef struct fs2_mt_state {
    uint32_t key[624];
    int32_t pos;
    int32_t has_gauss;
    double gauss;
} fs2_mt_state;
int fs2_mt_draw(fs2_handle *h, const fs2_mt_state *in, double sigma, fs2_mt_state *after,
                fs2_mt_state *after_u0, double *u0);
/* fs2_mt_draw in two halves around the next scan: the draw is enqueued here and
 * returns at once; the next fs2_iterate / fs2_iterate_submit ends it while its
 * candidate pass runs (the host's share of the draw -- the counts, the listed
 * logs, the patches -- then overlaps the GPU instead of preceding the scan) and
 * writes *after, *after_u0 and *u0 before it returns, whatever it returns; the
 * three must stay valid until then.  fs2_mt_draw, fs2_set_state, fs2_get_state
 * and fs2_debug_noise end a pending deferred draw first. */
int fs2_mt_draw_deferred(fs2_handle *h, const fs2_mt_state *in, double sigma, fs2_mt_state *after,
                         fs2_mt_state *after_u0, double *u0);

/* Particle state in the reference's object layout (Particle.x/.y/.yaw/.weight,
 * Particle.landmarks[j] = Landmark(x, y, cov) -- models/particle.py:11-20,
 * models/landmark.py:13-21).  Range [first, first+count) of this rank's local
 * particles.  lm is [count][lm_cap][6] = x, y, P00, P01, P10, P11; get_state
 * zero-fills slots beyond cnt[i].  where = FS2_HOST or FS2_DEVICE. Any of
 * x/y/yaw/w/cnt/lm may be NULL to skip it (set_state: cnt and lm go together). */
int fs2_get_state(fs2_handle *h, int64_t first, int64_t count, double *x, double *y,
                  double *yaw, double *w, int32_t *cnt, double *lm, int32_t lm_cap,
                  int32_t where);
int fs2_set_state(fs2_handle *h, int64_t first, int64_t count, const double *x,
                  const double *y, const double *yaw, const double *w, const int32_t *cnt,
                  const double *lm, int32_t lm_cap, int32_t where);

/* Association index per (measurement, local particle) of the last scan,
 * [M][N_local] row-major; -1 = no landmark associated (a new one was appended).
 * The particles are those of the scan's update pass, before its resample (a
 * sharded rank: the shard it held before the scan; see fs2_shard_info).
 * Mirrors the return of LandmarkUtils.associate_landmarks (landmark_utils.py:92-117).
 * Requires cfg.record_assoc. */
int fs2_get_assoc(fs2_handle *h, int32_t *idx, int64_t capacity, int32_t *m_out);

/* Local shard geometry and current map capacity.  With world_size > 1 and
 * num_particles divisible by world_size, a resample may hand this rank another
 * shard (the one its own sources fill most), so first_global can
 * change after any scan that resampled: read it after the scan, not once. */
int fs2_shard_info(const fs2_handle *h, int64_t *n_local, int64_t *first_global,
                   int32_t *capacity);

int fs2_synchronize(fs2_handle *h);

/* Device-event timing of the hot-path kernels (bench.py roofline): enable = 0
 * off, k >= 1 every k-th scan (the start / end events of a dispatch delay the next
 * dispatch by a few microseconds, so sampling keeps that out of most scans).
 * Resets the profile. */
int fs2_set_profiling(fs2_handle *h, int32_t enable);
int fs2_get_profile(const fs2_handle *h, fs2_profile *out);

/* ------------------------------------------------------ stateless helpers ---- */

/* Replaces ICP.get_transformation (algorithms/icp.py:13-57): exact nearest
 * neighbour (the brute-force / KD-tree result, lowest index on ties, through a
 * uniform grid over the target cloud), closed-form 2-D Kabsch, stop when
 * |prev - mean NN distance| < threshold.  R: 2x2 row-major, t: 2. */
int fs2_icp(int32_t device, const double *src, int32_t n_src, const double *tgt,
            int32_t n_tgt, int32_t max_iterations, double threshold, double R[4],
            double t[2], int32_t *iterations);

/* fs2_icp split in two for pipelining (Robot.get_transformation_icp,
 * robot.py:108-120, aligns scan s+1 to scan s; the alignment of the next scan
 * can run beside the filter update of this one): fs2_icp_submit copies the
 * clouds and enqueues the alignment on the device's ICP stream; fs2_icp_wait
 * blocks until ticket's alignment is done and returns fs2_icp's outputs.  At
 * most FS2_ICP_SLOTS tickets may be outstanding per device (FS2_ERR_STATE
 * beyond that, or for a ticket that is not outstanding). */
#define FS2_ICP_SLOTS 4
int fs2_icp_submit(int32_t device, const double *src, int32_t n_src, const double *tgt,
                   int32_t n_tgt, int32_t max_iterations, double threshold, int64_t *ticket);
int fs2_icp_wait(int32_t device, int64_t ticket, double R[4], double t[2], int32_t *iterations);

/* B independent alignments of P points each (src/tgt [B][P][2]); R [B][4],
 * t [B][2], iterations [B] (nullable).  where: FS2_HOST or FS2_DEVICE. */
int fs2_icp_batched(int32_t device, int32_t B, int32_t P, const double *src,
                    const double *tgt, int32_t max_iterations, double threshold, double *R,
                    double *t, int32_t *iterations, int32_t where);

/* Replaces ICP.best_fit_transform (algorithms/icp.py:60-90). */
int fs2_best_fit_transform(int32_t device, const double *src, const double *tgt, int32_t n,
                           double R[4], double t[2]);

/* Replaces LineFilter.filter (algorithms/line_filter.py:12-21): per-column
 * correlate1d with a symmetric Gaussian of 2*radius+1 taps, mode='reflect'.
 * taps as scipy builds them (fs2_gaussian_taps, or numpy in the shim). */
int fs2_line_filter(int32_t device, const double *points, int32_t n, const double *taps,
                    int32_t radius, double *out);

/* scipy.ndimage._gaussian_kernel1d(sigma, 0, int(truncate*sigma + 0.5)) with libm
 * exp; returns the radius, or -1 if more than max_taps taps would be needed. */
int32_t fs2_gaussian_taps(double sigma, double truncate, double *taps, int32_t max_taps);

/* Replaces LandmarkUtils.associate_landmarks (utils/landmark_utils.py:92-117) with
 * GeometryUtils.mahalanobis_distance (utils/geometry_utils.py:13-23): first j with
 * sqrt(d^T inv(P_j) d) < gate, d = observed - landmark_j; lm is [L][6].
 * *index = -1 when none (reference returns (None, None)). */
int fs2_associate(int32_t device, const double observed[2], const double *lm, int32_t L,
                  double gate, int32_t *index);

/* Replaces GeometryUtils.mahalanobis_distance (utils/geometry_utils.py:13-23) for K
 * pairs: out[k] = sqrt(d^T inv(cov_k) d), d = b_k - a_k.  a, b: [K][2]; cov: [K][4]
 * row-major.  FS2_ERR_LINALG if a covariance is singular. */
int fs2_mahalanobis(int32_t device, const double *a, const double *b, const double *cov,
                    int32_t K, double *out);

/* Test hooks of the device generator that replaces the reference's
 * np.random draws when rng="device" (fast_slam_2.py:79,81 motion noise, :183
 * resample start): Philox4x32-10 (Salmon et al., Random123) and the motion
 * sample's standard normals (Box-Muller on one Philox block per draw; particle
 * g of scan s draws normal (seed, stream = s, index = g), scaled by the noise).
 * fs2_debug_philox: n blocks, counter ctr[4 i .. 4 i + 3], key key[2 i, 2 i + 1]
 * -> out[4 i ..].  fs2_debug_normals: indices first .. first + n - 1 into out.
 * Host buffers. */
int fs2_debug_philox(int32_t device, int64_t n, const uint32_t *ctr, const uint32_t *key, uint32_t *out);
int fs2_debug_normals(int32_t device, uint64_t seed, uint64_t stream, uint64_t first, int64_t n,
                      double *out);
/* Test hook of fs2_mt_draw's log: out[k] = log(x[k]) rounded from double-double,
 * amb[k] = 1 where the host recomputes it (within 0.025 ulp of a midpoint);
 * on_host = 1 runs the same arithmetic on the CPU.  x in (0, 1), host buffers. */
int fs2_debug_mt_log(int32_t device, const double *x, int64_t n, double *out, int32_t *amb,
                     int32_t on_host);
/* Test hook of page_refs' fallback: this rank reports, at its first scan, that it
 * could not map its peers' pools (as without peer access between devices); the
 * mode then turns off on every rank (fs2_profile.page_refs = -1).  Before the
 * first scan only. */
int fs2_debug_refuse_peer_maps(fs2_handle *h);
/* Test hook of the in-place pools: on = 1 makes the next pool growth that must move
 * its reserved range fail right after the move (as a failing hipMemCreate / hipMemMap
 * would), so the allocate-and-copy fallback runs (fs2_iter_stats.pool_copies).
 * Process-wide, one-shot. */
int fs2_debug_vm_fail_after_relocate(int32_t on);
/* Test hook: the handle's motion-noise buffer (N_local values: the last scan's
 * injected draws, or fs2_mt_draw's) into out. */
int fs2_debug_noise(fs2_handle *h, double *out);
/* The source of each local output of the last resample (out[n_local]: >= 0 a
 * local source index, < 0 -(k+1) the k-th received particle); returns n_local
 * or a negative error.  For the drift study (scripts/drift_study.py). */
int64_t fs2_debug_out_src(fs2_handle *h, int32_t *out, int64_t capacity);
/* The weights of the current particle buffer set (other = 0) or of the other one
 * (other = 1: after a resampling scan, the sources' normalised weights the
 * resample read), n_local values.  For diagnosing the exact-order reductions. */
int fs2_debug_weights(fs2_handle *h, int32_t other, double *out);
/* Handles created with FS2_GUARD=1 in the environment follow every buffer
 * fs2_create allocates with a known pattern: the number of pattern bytes that
 * changed (a kernel wrote past a buffer's end), the first such buffer's name in
 * first_bad; 0 when clean or without FS2_GUARD.  Drains the handle's stream. */
int64_t fs2_debug_check_guards(fs2_handle *h, char *first_bad, int64_t len);
/* Test hook of fs2_mt_draw's jump-ahead: the stream words x[J + 1 .. J + 624]
 * after the key x[0 .. 624) (J >= 1), as the GF(2) combination of x[1 .. 20561)
 * given by x^J mod the characteristic polynomial (host arithmetic). */
int fs2_debug_mt_jump(const uint32_t key[624], uint64_t J, uint32_t out[624]);

/* ---------------------------------------------------------- multi-GPU ---- */

/* Replaces GeometryUtils.cluster_points (utils/geometry_utils.py:26-62), i.e.
 * sklearn DBSCAN(eps, min_samples) over n points (x, y) followed by the centre
 * (numpy mean) of every cluster, clusters in sklearn's label order.  Exact:
 * labels equal sklearn's (border points to the lowest-numbered cluster in reach).
 * centres is [cap][2]; K > cap sets *n_clusters = K and fails with FS2_ERR_ARG.
 * labels (nullable) receives n labels, -1 = noise.  where: FS2_HOST / FS2_DEVICE
 * for points, centres and labels.  Non-finite input fails (sklearn raises). */
int fs2_cluster_points(int32_t device, const double *points, int64_t n, double eps,
                       int64_t min_samples, double *centres, int64_t cap, int64_t *n_clusters,
                       int32_t *labels, int32_t where);

/* Replaces LandmarkUtils.update_known_landmarks (utils/landmark_utils.py:120-144)
 * for the particles held by the handle, without moving them off the device: every
 * landmark (x, y) in (particle, slot) order, min_samples = int(total / N *
 * min_fraction) (reference: 0.7), DBSCAN eps (reference: 0.5), centres in label
 * order into centres[cap][2] (host).  *n_clusters = -1 when min_samples < 1 (the
 * reference returns without updating).  Single-rank handles only. */
int fs2_update_known_landmarks(fs2_handle *h, double eps, double min_fraction, double *centres,
                               int64_t cap, int64_t *n_clusters);

/* ------------------------------------------- landmark front-end (§8f 1) ---- */

/* Outputs of fs2_frontend; every array is [B][cap][2] on the host and may be
 * NULL except counts.  Rows past a scan's count are left undefined. */
typedef struct fs2_frontend_out {
    int32_t cap;             /* rows per scan of each non-NULL array below */
    float *lines;            /* (rho, theta) in cv2.HoughLines order (hough_transformation.py:25) */
    double *intersections;   /* HoughTransformation.detect_line_intersections (hough_transformation.py:14-41) */
    double *clusters;        /* GeometryUtils.cluster_points(intersections, 0.5, 1) (landmark_utils.py:54-59) */
    double *corners;         /* LandmarkUtils.get_observed_landmarks (landmark_utils.py:39-64): (x, y) */
    double *measurements;    /* LandmarkUtils.get_measurements_to_landmarks (landmark_utils.py:21-36):
                                (distance, angle) = GeometryUtils.calculate_distance_and_angle */
    int32_t *counts;         /* [B][4]: lines, intersections, clusters, corners (required) */
} fs2_frontend_out;

/* Replaces LandmarkUtils.get_measurements_to_landmarks (utils/landmark_utils.py:21-89)
 * with LineFilter.filter (algorithms/line_filter.py:12-21), HoughTransformation
 * (algorithms/hough_transformation.py:14-145: image at 100 px/m, padding 20,
 * filled radius-2 circles, cv2.HoughLines(img, 1, pi/180, 80), pairwise
 * intersections of lines >= 45 deg apart), DBSCAN(eps 0.5, min_samples 1) means
 * and the 0.1 m corner test, for B scans in one call.  Scan b is points
 * [offsets[b], offsets[b+1]) of points[][2] (x, y); offsets: host, B + 1 entries.
 * taps/radius: the LineFilter Gaussian (fs2_gaussian_taps; sigma 0.1 gives the
 * identity, radius 0).  legacy = 0 follows numpy >= 2 scalar promotion (float32
 * intersections, centres and corners; what the fixtures pin), 1 numpy 1.x
 * (float64 from the back-conversion on).  where: FS2_HOST / FS2_DEVICE for points.
 * FS2_ERR_ARG for an empty or non-finite scan (the reference raises ValueError),
 * an image over 20000 px in width + height, more than 4096 Hough lines in a
 * scan, or a count above out->cap for a requested array (counts still filled). */
int fs2_frontend(int32_t device, int32_t B, const int64_t *offsets, const double *points,
                 int32_t where, const double *taps, int32_t radius, int32_t legacy,
                 fs2_frontend_out *out);

/* ncclUniqueId for fs2_config.comm_id (call on rank 0, broadcast to all ranks). */
int fs2_comm_unique_id(uint8_t out[128]);

/* The sharded low-variance resample plan of one rank (replaces the loop of
 * FastSLAM2.__low_variance_resample, algorithms/fast_slam_2.py:177-199, for the
 * rank's particles; csrc/fs2_plan.hpp), on the host with the arithmetic the
 * device kernels k_ranges / k_pack_bounds run, for callers that plan transfers
 * themselves and for the CPU tests.  Host pointers.
 * fs2_plan_ranges: the output range [mlo[i], mhi[i]] (empty when mlo > mhi) of
 *   local particle i (global first_global + i) from the local inclusive prefix
 *   c[0..n) of the normalised weights, the sum `offset` of the earlier ranks'
 *   totals (0 on rank 0) and the start u0; outputs follow u_m = u0 + m (1/N).
 * fs2_plan_sends: for every rank p of `world` (shard [N p / world, N (p+1) / world)),
 *   the run [run[2p], run[2p+1]) of local particles whose ranges reach that shard
 *   and the K[p] particles (non-empty ranges) and S[p] map slots (cnt) this rank
 *   sends it (0 for p == rank). */
int fs2_plan_ranges(const double *c, int64_t n, int64_t first_global, int64_t N, double offset, double u0,
                    int32_t *mlo, int32_t *mhi);
int fs2_plan_sends(const int32_t *mlo, const int32_t *mhi, const int32_t *cnt, int64_t n, int64_t N,
                   int32_t world, int32_t rank, int64_t *run, int64_t *K, int64_t *S);

#ifdef __cplusplus
}
#endif

#endif /* FS2_H */
