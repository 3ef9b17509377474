// fs2_kernels.hip -- CDNA4 (gfx950) kernels of the FastSLAM 2.0 particle update.
//
// Layout in HBM: particle SoA x/y/yaw/w (fp64) + cnt (int32);
// landmark maps in pages of 64 slots, each slot three double2 planes over the
// particles -- plane 0 (x, y), plane 1 (P00, P01), plane 2 (P10, P11) -- so a
// wave reading one slot of 64 consecutive particles issues three fully
// coalesced 1 KiB loads.
//
// Kernels
//   k_update      fused move + association + EKF/append + likelihood, ONE pass
//                 over each particle's map for up to kMaxM measurements
//                 (fast_slam_2.py:33-159);
//   k_wsum        weight total (fast_slam_2.py:166);
//   k_normalize   normalise + per-block sum w'^2 / argmax / max count (:161-175);
//   k_finalize    N_eff, resample decision, estimate, u0 (:60-67, :201-223);
//   k_scan_*, k_resample_src, k_gather_*, k_estimate   low-variance resample (:177-199);
//   k_icp         one workgroup per alignment (icp.py:13-90);
//   k_line_filter, k_associate, k_import/k_export.
#include "fs2_device.hpp"
#include "fs2_kernels.hpp"

namespace fs2 {

// ------------------------------------------------------------ reductions ---

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// (value, index) argmax, lowest index among equal maxima (Python max).
__device__ __forceinline__ void argmax_combine(double &v, int64_t &i, double v2, int64_t i2) {
    if (v2 > v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

__device__ __forceinline__ void wave_argmax(double &v, int64_t &i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double v2 = __shfl_xor(v, o, 64);
        const int64_t i2 = __shfl_xor(i, o, 64);
        argmax_combine(v, i, v2, i2);
    }
}

// Deterministic block sum (fixed tree), result valid in every thread.
template <int NT>
__device__ double block_sum(double v, double *lds) {
    v = wave_sum(v);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) t += lds[k];
    return t;
}

template <int NT>
__device__ unsigned long long block_sum_u64(unsigned long long v, unsigned long long *lds) {
    v = wave_sum_u64(v);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    unsigned long long t = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) t += lds[k];
    return t;
}

template <int NT>
__device__ void block_argmax(double &v, int64_t &i, double *ldv, int64_t *ldi) {
    wave_argmax(v, i);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) {
        ldv[wid] = v;
        ldi[wid] = i;
    }
    __syncthreads();
    v = ldv[0];
    i = ldi[0];
#pragma unroll
    for (int k = 1; k < NT / 64; ++k) argmax_combine(v, i, ldv[k], ldi[k]);
}

template <int NT>
__device__ int block_max_i(int v, int *lds) {
    v = wave_max_i(v);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    int t = lds[0];
#pragma unroll
    for (int k = 1; k < NT / 64; ++k) t = max(t, lds[k]);
    return t;
}

// ------------------------------------------------------------- map access ---

__device__ __forceinline__ const double2 *slot_planes(const MapRef &m, int j) {
    return reinterpret_cast<const double2 *>(m.pages[j >> 6] +
                                             (int64_t)(j & (kPageSlots - 1)) * m.slot_stride());
}

__device__ __forceinline__ Slot load_slot(const MapRef &m, int j, int64_t i) {
    const double2 *p = slot_planes(m, j);
    const double2 a = p[i], b = p[m.n + i], c = p[2 * m.n + i];
    return Slot{a.x, a.y, M2{b.x, b.y, c.x, c.y}};
}

__device__ __forceinline__ float4 load_mirror(const MapRef &m, int j, int64_t i) {
    return reinterpret_cast<const float4 *>(slot_planes(m, j) + kMirrorPlane * m.n)[i];
}

// Every slot write keeps the fp32 gate mirror in step with the fp64 slot.
__device__ __forceinline__ void store_slot(const MapRef &m, int j, int64_t i, const Slot &s) {
    double2 *p = const_cast<double2 *>(slot_planes(m, j));
    p[i] = make_double2(s.mx, s.my);
    p[m.n + i] = make_double2(s.P.a00, s.P.a01);
    p[2 * m.n + i] = make_double2(s.P.a10, s.P.a11);
    reinterpret_cast<float4 *>(p + kMirrorPlane * m.n)[i] = mirror_of(s);
}

// Gate decisions this close to the threshold could depend on ulp-level
// differences upstream (landmark means after EKF); counted, never altered.
__device__ __forceinline__ unsigned ambiguous(double q, double gate2) {
    return fabs(q - gate2) <= 1e-9 * gate2 ? 1u : 0u;
}

// ------------------------------------------------------------ k_update ------
//
// One lane per particle.  The M measurements of a scan are sequential in the
// reference (measurement k sees the map left by k-1), but measurement k only
// ever changes the slot it matched or appends at the end.  Walking the map
// once and, at every slot j, testing the still-unmatched measurements in
// order k = 0..M-1 (an EKF update changes the slot in registers before the
// next measurement tests it) reproduces the sequential result exactly while
// reading each slot once instead of M times.  Slots appended in this scan are
// resolved afterwards in measurement order.  Likelihoods multiply into the
// weight in measurement order, as the reference does.
template <int MAXM>
__global__ __launch_bounds__(kBlock) void k_update(const UpdateParams P) {
    __shared__ double lds_d[kBlock / 64];
    __shared__ unsigned long long lds_u[kBlock / 64];
    __shared__ int lds_i[kBlock / 64];
    __shared__ Meas s_ms[MAXM];                 // this pass's measurements
    __shared__ double s_lik[MAXM][kBlock];      // per (measurement, lane) likelihood
    __shared__ int s_idx[MAXM][kBlock];         // per (measurement, lane) association

    const int tid = threadIdx.x;
    const int64_t i = (int64_t)blockIdx.x * kBlock + tid;
    const bool live = i < P.n;
    const int64_t n = P.n;
    if (tid < MAXM) s_ms[tid] = Meas{P.meas.d[tid], P.meas.b[tid], P.meas.ox[tid], P.meas.oy[tid]};
#pragma unroll
    for (int k = 0; k < MAXM; ++k) s_idx[k][tid] = -2;
    __syncthreads();

    double px = 0.0, py = 0.0, pyaw = 0.0, w = 0.0;
    int c = 0;
    if (live) {
        px = P.x[i];
        py = P.y[i];
        pyaw = P.yaw[i];
        w = P.w[i];
        c = P.cnt[i];
    }
    // __move_particle (fast_slam_2.py:69-87)
    if (live && P.do_move) {
        const double nz = P.noise ? P.noise[i]
                                  : P.sigma * philox_normal(P.seed, P.scan, (uint64_t)(P.gidx0 + i));
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

    const M2 R{P.R[0], P.R[1], P.R[2], P.R[3]};
    unsigned pend = live ? ((1u << P.m) - 1u) : 0u;
    unsigned visited = 0, written = 0, amb = 0, appends = 0;
    bool singular = false;
    const double gate2 = P.gate2;

    // ---- single pass over the existing map (association + EKF) ----
    // Steps of kGroup slots: the fp32 mirrors of the whole group are loaded
    // first (1 KiB per wave and slot, all in flight together); a slot whose
    // mirror cannot rule out every still-pending measurement becomes a
    // candidate and takes the exact fp64 path, in slot order.
    unsigned candidates = 0;
    for (int j0 = 0;; j0 += kGroup) {
        if (!__any((pend != 0u) && (j0 < c))) break;
        unsigned cmask = 0;
        if (P.filter) {
            float4 mir[kGroup];
#pragma unroll
            for (int u = 0; u < kGroup; ++u)
                if (pend != 0u && j0 + u < c) mir[u] = load_mirror(P.map, j0 + u, i);
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                if (pend != 0u && j0 + u < c) {
                    ++visited;
                    bool cand = false;
#pragma unroll
                    for (int k = 0; k < MAXM; ++k)
                        if ((pend >> k) & 1u)
                            cand |= !gate_reject(mir[u], P.meas.fx[k], P.meas.fy[k], P.meas.fe[k],
                                                 P.gate2f);
                    if (cand) cmask |= 1u << u;
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < kGroup; ++u)
                if (pend != 0u && j0 + u < c) {
                    ++visited;
                    cmask |= 1u << u;
                }
        }
        while (cmask) {
            const int j = j0 + __builtin_ctz(cmask);
            cmask &= cmask - 1u;
            if (pend == 0u) break;
            Slot s = load_slot(P.map, j, i);
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
                        const double q = quad(I, s_ms[k].ox - s.mx, s_ms[k].oy - s.my);
                        amb += ambiguous(q, gate2);
                        todo &= ~(1u << k);
                        if (q >= 0.0 && q < gate2) km = k;
                    }
                }
                if (km < 0) break;
                // one EKF site: the matched measurement sees the slot as left by
                // the earlier measurements (fast_slam_2.py:116-153)
                s_lik[km][tid] = ekf_update(s, px, py, pyaw, s_ms[km], R, singular);
                s_idx[km][tid] = j;
                pend &= ~(1u << km);
                mod = true;
                ok = inv2(s.P, I);
                singular |= !ok;
                if (!ok) todo = 0u;
            }
            if (mod) {
                store_slot(P.map, j, i, s);
                ++written;
            }
        }
    }

    // ---- measurements that matched nothing: appended slots, in order ----
    int nap = 0;
    while (pend) {
        const int k = __builtin_ctz(pend);
        pend &= pend - 1u;
        const Meas mk = s_ms[k];
        int hit = -1;
        for (int a = 0; a < nap; ++a) {
            const Slot s = load_slot(P.map, c + a, i);
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
            Slot s = load_slot(P.map, c + hit, i);
            s_lik[k][tid] = ekf_update(s, px, py, pyaw, mk, R, singular);
            store_slot(P.map, c + hit, i, s);
            s_idx[k][tid] = c + hit;
        } else {
            // new landmark in the world frame (fast_slam_2.py:108-111)
            const Slot s{px + mk.d * cos(pyaw + mk.b), py + mk.d * sin(pyaw + mk.b),
                         M2{P.init_cov[0], P.init_cov[1], P.init_cov[2], P.init_cov[3]}};
            store_slot(P.map, c + nap, i, s);
            s_idx[k][tid] = -1;
            ++nap;
            ++appends;
        }
        ++written;
    }
    c += nap;

    // likelihoods in measurement order (fast_slam_2.py:159)
    unsigned hits = 0;
#pragma unroll
    for (int k = 0; k < MAXM; ++k) {
        const int ix = s_idx[k][tid];
        if (ix >= 0) {
            w *= s_lik[k][tid];
            ++hits;
        }
        if (live && P.assoc && k < P.m) P.assoc[(int64_t)(P.k0 + k) * n + i] = ix;
    }

    if (live) {
        if (P.do_move) {
            P.x[i] = px;
            P.y[i] = py;
            P.yaw[i] = pyaw;
        }
        P.w[i] = w;
        P.cnt[i] = c;
    }

    // ---- block statistics ----
    const unsigned long long bv = block_sum_u64<kBlock>(visited, lds_u);
    const unsigned long long bc = block_sum_u64<kBlock>(candidates, lds_u);
    const unsigned long long bw = block_sum_u64<kBlock>(written, lds_u);
    const unsigned long long ba = block_sum_u64<kBlock>(amb, lds_u);
    const unsigned long long bap = block_sum_u64<kBlock>(appends, lds_u);
    const unsigned long long bh = block_sum_u64<kBlock>(hits, lds_u);
    const int anysing = __syncthreads_or(singular ? 1 : 0);
    if (P.last_pass) {
        const double ws = block_sum<kBlock>(live ? w : 0.0, lds_d);
        const int mc = block_max_i<kBlock>(live ? c : 0, lds_i);
        if (tid == 0) {
            P.wpart[blockIdx.x] = ws;
            atomicMax(&P.stats->max_count, mc);
        }
    }
    if (tid == 0) {
        atomicAdd(&P.stats->visited, bv);
        atomicAdd(&P.stats->candidates, bc);
        atomicAdd(&P.stats->written, bw);
        atomicAdd(&P.stats->ambiguous, ba);
        atomicAdd(&P.stats->appends, bap);
        atomicAdd(&P.stats->hits, bh);
        if (anysing) atomicOr(&P.stats->error_flags, 1);
    }
}

hipError_t launch_update(const UpdateParams &p, hipStream_t s) {
    const unsigned grid = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_update<kMaxM>, dim3(grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------- normalise & N_eff --

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
    // iterative split (numpy recursion), at most log2(8192/128)+1 levels deep
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sq(a, n2) + pairwise_sq(a + n2, n - n2);
}

// Weight total. Sequential mode: Python builtin sum in particle order.
__global__ __launch_bounds__(1024) void k_wsum(const ReduceParams P) {
    __shared__ double lds[16];
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

hipError_t launch_wsum(const ReduceParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_wsum, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_normalize(const ReduceParams P) {
    __shared__ double lds_d[kBlock / 64];
    __shared__ int64_t lds_l[kBlock / 64];
    __shared__ int lds_i[kBlock / 64];
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
    const double sq = block_sum<kBlock>(live ? w * w : 0.0, lds_d);
    double bv = live ? w : -INFINITY;
    int64_t bi = live ? i : INT64_MAX;
    block_argmax<kBlock>(bv, bi, lds_d, lds_l);
    const int mc = block_max_i<kBlock>(c, lds_i);
    if (threadIdx.x == 0) {
        P.part_sq[blockIdx.x] = sq;
        P.part_best_w[blockIdx.x] = bv;
        P.part_best_i[blockIdx.x] = bi;
        P.part_maxcnt[blockIdx.x] = mc;
    }
}

hipError_t launch_normalize(const ReduceParams &p, hipStream_t s) {
    const unsigned grid = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_normalize, dim3(grid), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

// N_eff, resample decision, estimate (pre-resample), u0.
__global__ __launch_bounds__(1024) void k_finalize(const ReduceParams P) {
    __shared__ double lds_d[16];
    __shared__ int64_t lds_l[16];
    __shared__ int lds_i[16];
    double sq = 0.0;
    double bv = -INFINITY;
    int64_t bi = INT64_MAX;
    int mc = 0;
    for (int k = threadIdx.x; k < P.nparts; k += 1024) {
        sq += P.part_sq[k];
        argmax_combine(bv, bi, P.part_best_w[k], P.part_best_i[k]);
        mc = max(mc, P.part_maxcnt[k]);
    }
    sq = block_sum<1024>(sq, lds_d);
    block_argmax<1024>(bv, bi, lds_d, lds_l);
    mc = block_max_i<1024>(mc, lds_i);
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
        }
        const double ng = (double)P.n_global;
        const double ne = (sq < 1.0 / ng) ? ng : 1.0 / sq;
        DevStats *st = P.stats;
        st->sumsq = sq;
        st->n_eff = ne;
        st->resampled = ne < ng / 2.0 ? 1 : 0;
        st->max_count = max(st->max_count, mc);
        st->best_index = bi;
        st->best_w = bv;
        st->pose[0] = P.x[bi];
        st->pose[1] = P.y[bi];
        st->pose[2] = P.yaw[bi];
        const double r = P.u0_host ? *P.u0_host
                                   : (1.0 / ng) * philox_uniform01(P.seed, P.scan | (1ull << 63), 0);
        st->u0 = r;
    }
}

hipError_t launch_finalize(const ReduceParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}

// -------------------------------------------------------------- resample ---

constexpr int kScanPer = 4;                       // elements per thread
constexpr int kScanBlock = kBlock * kScanPer;     // 1024 elements per block

__global__ __launch_bounds__(1) void k_scan_seq(const ResampleParams P) {
    if (!P.stats->resampled) return;
    double c = 0.0;
    for (int64_t i = 0; i < P.n; ++i) {
        c = (i == 0) ? P.w[0] : c + P.w[i];
        P.c[i] = c;
    }
}

__device__ __forceinline__ double wave_incl_scan(double v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__global__ __launch_bounds__(kBlock) void k_scan_local(const ResampleParams P) {
    __shared__ double lds[kBlock / 64];
    if (!P.stats->resampled) return;
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

__global__ __launch_bounds__(1) void k_scan_blocks(const ResampleParams P) {
    if (!P.stats->resampled) return;
    double acc = 0.0;
    for (int b = 0; b < P.nblk; ++b) {
        const double t = P.bsum[b];
        P.bsum[b] = acc;    // exclusive offset
        acc += t;
    }
}

__global__ __launch_bounds__(kBlock) void k_scan_add(const ResampleParams P) {
    if (!P.stats->resampled) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < P.n) P.c[i] += P.bsum[i / kScanBlock];
}

// src(m) = smallest i with prefix c_i >= u_m, else N-1 (fast_slam_2.py:188-196,
// without the reference's hang when u_m exceeds every reachable sum, Q10).
__global__ __launch_bounds__(kBlock) void k_resample_src(const ResampleParams P) {
    if (!P.stats->resampled) return;
    const int64_t m = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (m >= P.n) return;
    const double u = P.stats->u0 + (double)m * (1.0 / (double)P.n);
    int64_t lo = 0, hi = P.n;   // first index with c >= u in [lo, hi)
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (P.c[mid] >= u) hi = mid;
        else lo = mid + 1;
    }
    P.src[m] = (lo < P.n) ? (int32_t)lo : (int32_t)(P.n - 1);
}

__global__ __launch_bounds__(kBlock) void k_gather_particles(const ResampleParams P) {
    __shared__ double lds_d[kBlock / 64];
    __shared__ int64_t lds_l[kBlock / 64];
    if (!P.stats->resampled) return;
    const int64_t m = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double bv = -INFINITY;
    int64_t bi = INT64_MAX;
    if (m < P.n) {
        const int32_t s = P.src[m];
        P.ox[m] = P.x[s];
        P.oy[m] = P.y[s];
        P.oyaw[m] = P.yaw[s];
        const double w = P.w[s];
        P.ow[m] = w;
        P.ocnt[m] = P.cnt[s];
        bv = w;
        bi = m;
    }
    block_argmax<kBlock>(bv, bi, lds_d, lds_l);
    if (threadIdx.x == 0) {
        P.part_best_w[blockIdx.x] = bv;
        P.part_best_i[blockIdx.x] = bi;
    }
}

constexpr int kGatherSlots = 16;   // slots per thread in the map gather

// Deep copy of the selected maps (fast_slam_2.py:196): blockIdx.y picks a
// chunk of 16 slots, lanes run over output particles (coalesced writes; the
// monotone src keeps reads nearly coalesced).
__global__ __launch_bounds__(kBlock) void k_gather_maps(const ResampleParams P) {
    __shared__ unsigned long long lds_u[kBlock / 64];
    if (!P.stats->resampled) return;
    const int64_t m = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int j0 = blockIdx.y * kGatherSlots;
    unsigned long long copied = 0;
    if (m < P.n) {
        const int32_t s = P.src[m];
        const int cnt = P.cnt[s];
        const int jend = min(cnt, j0 + kGatherSlots);
        for (int j = j0; j < jend; ++j) {
            const double2 *ip = slot_planes(P.in, j);
            double2 *op = const_cast<double2 *>(slot_planes(P.out, j));
            const double2 a = ip[s], b = ip[P.in.n + s], c = ip[2 * P.in.n + s];
            const double2 g = ip[kMirrorPlane * P.in.n + s];   // gate mirror (16 B)
            op[m] = a;
            op[P.out.n + m] = b;
            op[2 * P.out.n + m] = c;
            op[kMirrorPlane * P.out.n + m] = g;
            ++copied;
        }
    }
    const unsigned long long bc = block_sum_u64<kBlock>(copied, lds_u);
    if (threadIdx.x == 0 && bc) atomicAdd(&P.stats->resample_slots, bc);
}

__global__ __launch_bounds__(1024) void k_estimate(const ResampleParams P, int32_t nparts) {
    __shared__ double lds_d[16];
    __shared__ int64_t lds_l[16];
    if (!P.stats->resampled) return;
    double bv = -INFINITY;
    int64_t bi = INT64_MAX;
    for (int k = threadIdx.x; k < nparts; k += 1024) argmax_combine(bv, bi, P.part_best_w[k], P.part_best_i[k]);
    block_argmax<1024>(bv, bi, lds_d, lds_l);
    if (threadIdx.x == 0) {
        DevStats *st = P.stats;
        st->best_index = bi;
        st->best_w = bv;
        st->pose[0] = P.ox[bi];
        st->pose[1] = P.oy[bi];
        st->pose[2] = P.oyaw[bi];
    }
}

hipError_t launch_resample(const ResampleParams &p, int sequential, int32_t cap, hipStream_t s) {
    const unsigned g = (unsigned)((p.n + kBlock - 1) / kBlock);
    if (g == 0) return hipSuccess;
    if (sequential) {
        hipLaunchKernelGGL(k_scan_seq, dim3(1), dim3(1), 0, s, p);
    } else {
        hipLaunchKernelGGL(k_scan_local, dim3(p.nblk), dim3(kBlock), 0, s, p);
        hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1), 0, s, p);
        hipLaunchKernelGGL(k_scan_add, dim3(g), dim3(kBlock), 0, s, p);
    }
    hipLaunchKernelGGL(k_resample_src, dim3(g), dim3(kBlock), 0, s, p);
    hipLaunchKernelGGL(k_gather_particles, dim3(g), dim3(kBlock), 0, s, p);
    const unsigned gy = (unsigned)((cap + kGatherSlots - 1) / kGatherSlots);
    if (gy) hipLaunchKernelGGL(k_gather_maps, dim3(g, gy), dim3(kBlock), 0, s, p);
    hipLaunchKernelGGL(k_estimate, dim3(1), dim3(1024), 0, s, p, (int32_t)g);
    return hipGetLastError();
}

// ------------------------------------------------------ state import/export --

// stage: [count][lm_cap][6] -> pages; cnt_stage: [count]
__global__ __launch_bounds__(kBlock) void k_import(const double *stage, const int32_t *cnt_stage,
                                                   int64_t first, int64_t count, int32_t lm_cap,
                                                   MapRef map, int32_t *cnt) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t total = count * lm_cap;
    for (int64_t e = t; e < total; e += (int64_t)gridDim.x * kBlock) {
        const int64_t p = e / lm_cap;
        const int j = (int)(e % lm_cap);
        const int c = cnt_stage[p];
        if (j == 0) cnt[first + p] = c;
        if (j >= c) continue;
        const double *s = stage + e * 6;
        store_slot(map, j, first + p, Slot{s[0], s[1], M2{s[2], s[3], s[4], s[5]}});
    }
}

__global__ __launch_bounds__(kBlock) void k_export(double *stage, int64_t first, int64_t count,
                                                   int32_t lm_cap, MapRef map, const int32_t *cnt) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t total = count * lm_cap;
    for (int64_t e = t; e < total; e += (int64_t)gridDim.x * kBlock) {
        const int64_t p = e / lm_cap;
        const int j = (int)(e % lm_cap);
        if (j >= cnt[first + p]) continue;
        const Slot s = load_slot(map, j, first + p);
        double *d = stage + e * 6;
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
                         int64_t count, int32_t lm_cap, MapRef map, int32_t *cnt, hipStream_t s) {
    hipLaunchKernelGGL(k_import, dim3(grid_for(count * lm_cap)), dim3(kBlock), 0, s, stage,
                       cnt_stage, first, count, lm_cap, map, cnt);
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

// ------------------------------------------------------------------- ICP ---
//
// One workgroup per alignment; the target cloud and the moving source cloud
// live in LDS for the whole loop; nearest neighbours by brute force with
// broadcast LDS reads (every lane reads the same target point), lowest index
// on exact ties; centroids / cross-covariance / mean distance by fixed-order
// wave + LDS reductions; rotation by the closed-form 2-D Kabsch angle, which
// equals the reference's SVD + reflection fix (icp.py:76-85).

constexpr int kIcpMaxP = 1024;
constexpr int kIcpThreads = 1024;

template <int NT>
__device__ void block_sum5(double v[5], double *lds) {
#pragma unroll
    for (int q = 0; q < 5; ++q) v[q] = wave_sum(v[q]);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 5; ++q) lds[q * 16 + wid] = v[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < NT / 64; ++k) t += lds[q * 16 + k];
        v[q] = t;
    }
}

__global__ __launch_bounds__(kIcpThreads) void k_icp(int32_t P, const double *src_all,
                                                     const double *tgt_all, int32_t nt,
                                                     int32_t max_iter, double thr, double *R_out,
                                                     double *t_out, int32_t *iters_out) {
    __shared__ double2 s_src[kIcpMaxP];
    __shared__ double2 s_tgt[kIcpMaxP];
    __shared__ int32_t s_nn[kIcpMaxP];
    __shared__ double s_dist[kIcpMaxP];
    __shared__ double red[5 * 16];
    __shared__ double s_R[4], s_t[2];
    __shared__ int s_stop;

    const int b = blockIdx.x;
    const double2 *src = reinterpret_cast<const double2 *>(src_all) + (int64_t)b * P;
    const double2 *tgt = reinterpret_cast<const double2 *>(tgt_all) + (int64_t)b * nt;
    for (int k = threadIdx.x; k < P; k += kIcpThreads) s_src[k] = src[k];
    for (int k = threadIdx.x; k < nt; k += kIcpThreads) s_tgt[k] = tgt[k];
    double Rt[4] = {1.0, 0.0, 0.0, 1.0}, tt[2] = {0.0, 0.0};
    double prev = INFINITY;
    int it = 0;
    __syncthreads();
    while (it < max_iter) {
        ++it;
        // nearest neighbours
        for (int k = threadIdx.x; k < P; k += kIcpThreads) {
            const double2 sp = s_src[k];
            double best = INFINITY;
            int bj = 0;
            for (int j = 0; j < nt; ++j) {
                const double2 tp = s_tgt[j];
                const double dx = sp.x - tp.x, dy = sp.y - tp.y;
                const double d2 = dx * dx + dy * dy;
                if (d2 < best) {
                    best = d2;
                    bj = j;
                }
            }
            s_nn[k] = bj;
            s_dist[k] = sqrt(best);
        }
        __syncthreads();
        // centroids and mean distance
        double v[5] = {0, 0, 0, 0, 0};
        for (int k = threadIdx.x; k < P; k += kIcpThreads) {
            const double2 sp = s_src[k], tp = s_tgt[s_nn[k]];
            v[0] += sp.x; v[1] += sp.y; v[2] += tp.x; v[3] += tp.y; v[4] += s_dist[k];
        }
        block_sum5<kIcpThreads>(v, red);
        const double cs0 = v[0] / P, cs1 = v[1] / P, ct0 = v[2] / P, ct1 = v[3] / P;
        const double mean = v[4] / P;
        // cross-covariance of the centred sets (icp.py:73)
        double h[5] = {0, 0, 0, 0, 0};
        for (int k = threadIdx.x; k < P; k += kIcpThreads) {
            const double2 sp = s_src[k], tp = s_tgt[s_nn[k]];
            const double a0 = sp.x - cs0, a1 = sp.y - cs1, b0 = tp.x - ct0, b1 = tp.y - ct1;
            h[0] += a0 * b0; h[1] += a0 * b1; h[2] += a1 * b0; h[3] += a1 * b1;
        }
        block_sum5<kIcpThreads>(h, red);
        if (threadIdx.x == 0) {
            const double th = atan2(h[1] - h[2], h[0] + h[3]);
            const double c = cos(th), s = sin(th);
            const M2 Ri{c, -s, s, c};
            const double t0 = ct0 - fma(Ri.a00, cs0, Ri.a01 * cs1);
            const double t1 = ct1 - fma(Ri.a10, cs0, Ri.a11 * cs1);
            s_R[0] = Ri.a00; s_R[1] = Ri.a01; s_R[2] = Ri.a10; s_R[3] = Ri.a11;
            s_t[0] = t0; s_t[1] = t1;
            s_stop = fabs(prev - mean) < thr ? 1 : 0;
        }
        __syncthreads();
        const double r00 = s_R[0], r01 = s_R[1], r10 = s_R[2], r11 = s_R[3], t0 = s_t[0], t1 = s_t[1];
        for (int k = threadIdx.x; k < P; k += kIcpThreads) {
            const double2 sp = s_src[k];
            s_src[k] = make_double2(fma(sp.y, r01, sp.x * r00) + t0, fma(sp.y, r11, sp.x * r10) + t1);
        }
        const M2 Rn = mm2(M2{r00, r01, r10, r11}, M2{Rt[0], Rt[1], Rt[2], Rt[3]});
        Rt[0] = Rn.a00; Rt[1] = Rn.a01; Rt[2] = Rn.a10; Rt[3] = Rn.a11;
        const double nt0 = fma(r00, tt[0], r01 * tt[1]) + t0;
        const double nt1 = fma(r10, tt[0], r11 * tt[1]) + t1;
        tt[0] = nt0;
        tt[1] = nt1;
        const int stop = s_stop;
        prev = mean;
        __syncthreads();
        if (stop) break;
    }
    if (threadIdx.x == 0) {
        for (int q = 0; q < 4; ++q) R_out[b * 4 + q] = Rt[q];
        t_out[b * 2] = tt[0];
        t_out[b * 2 + 1] = tt[1];
        if (iters_out) iters_out[b] = it;
    }
}

hipError_t launch_icp(int32_t B, int32_t P, const double *src, const double *tgt, int32_t n_tgt,
                      int32_t max_iter, double thr, double *R, double *t, int32_t *iters,
                      double *scratch, hipStream_t s) {
    (void)scratch;
    if (P > kIcpMaxP || n_tgt > kIcpMaxP) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_icp, dim3(B), dim3(kIcpThreads), 0, s, P, src, tgt, n_tgt, max_iter, thr,
                       R, t, iters);
    return hipGetLastError();
}

// best_fit_transform alone: Rt = [R00 R01 R10 R11 t0 t1]
__global__ __launch_bounds__(kIcpThreads) void k_best_fit(const double *src_, const double *tgt_,
                                                          int32_t P, double *Rt) {
    __shared__ double red[5 * 16];
    const double2 *src = reinterpret_cast<const double2 *>(src_);
    const double2 *tgt = reinterpret_cast<const double2 *>(tgt_);
    double v[5] = {0, 0, 0, 0, 0};
    for (int k = threadIdx.x; k < P; k += kIcpThreads) {
        v[0] += src[k].x; v[1] += src[k].y; v[2] += tgt[k].x; v[3] += tgt[k].y;
    }
    block_sum5<kIcpThreads>(v, red);
    const double cs0 = v[0] / P, cs1 = v[1] / P, ct0 = v[2] / P, ct1 = v[3] / P;
    double h[5] = {0, 0, 0, 0, 0};
    for (int k = threadIdx.x; k < P; k += kIcpThreads) {
        const double a0 = src[k].x - cs0, a1 = src[k].y - cs1, b0 = tgt[k].x - ct0, b1 = tgt[k].y - ct1;
        h[0] += a0 * b0; h[1] += a0 * b1; h[2] += a1 * b0; h[3] += a1 * b1;
    }
    block_sum5<kIcpThreads>(h, red);
    if (threadIdx.x == 0) {
        const double th = atan2(h[1] - h[2], h[0] + h[3]);
        const double c = cos(th), s = sin(th);
        Rt[0] = c; Rt[1] = -s; Rt[2] = s; Rt[3] = c;
        Rt[4] = ct0 - fma(c, cs0, -s * cs1);
        Rt[5] = ct1 - fma(s, cs0, c * cs1);
    }
}

hipError_t launch_best_fit(const double *src, const double *tgt, int32_t n, double *Rt, hipStream_t s) {
    hipLaunchKernelGGL(k_best_fit, dim3(1), dim3(kIcpThreads), 0, s, src, tgt, n, Rt);
    return hipGetLastError();
}

// ------------------------------------------------------------ LineFilter ---

__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t n) {
    const int64_t p = 2 * n;
    int64_t k = i % p;
    if (k < 0) k += p;
    return (k < n) ? k : p - 1 - k;
}

// scipy correlate1d, symmetric kernel branch, mode='reflect' (ni_filters.c
// order: centre tap first, then (x[i-k] + x[i+k]) * w for k = r..1).
__global__ __launch_bounds__(kBlock) void k_line_filter(const double *in, int32_t n,
                                                        const double *taps, int32_t r,
                                                        double *out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= 2 * (int64_t)n) return;
    const int64_t i = e >> 1;
    const int col = (int)(e & 1);
    double acc = in[reflect_idx(i, n) * 2 + col] * taps[r];
    for (int jj = -r; jj < 0; ++jj)
        acc += (in[reflect_idx(i + jj, n) * 2 + col] + in[reflect_idx(i - jj, n) * 2 + col]) * taps[r + jj];
    out[e] = acc;
}

hipError_t launch_line_filter(const double *in, int32_t n, const double *taps, int32_t r,
                              double *out, hipStream_t s) {
    const unsigned g = (unsigned)((2 * (int64_t)n + kBlock - 1) / kBlock);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(k_line_filter, dim3(g), dim3(kBlock), 0, s, in, n, taps, r, out);
    return hipGetLastError();
}

// ----------------------------------------------------------- mahalanobis ---
__global__ __launch_bounds__(kBlock) void k_mahalanobis(const double *a, const double *b,
                                                        const double *cov, int32_t K, double *out,
                                                        int32_t *singular) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= K) return;
    M2 I;
    if (!inv2(M2{cov[4 * k], cov[4 * k + 1], cov[4 * k + 2], cov[4 * k + 3]}, I)) {
        atomicOr(singular, 1);
        out[k] = NAN;
        return;
    }
    out[k] = sqrt(quad(I, b[2 * k] - a[2 * k], b[2 * k + 1] - a[2 * k + 1]));
}

hipError_t launch_mahalanobis(const double *a, const double *b, const double *cov, int32_t K,
                              double *out, int32_t *singular, hipStream_t s) {
    const unsigned g = (unsigned)((K + kBlock - 1) / kBlock);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mahalanobis, dim3(g), dim3(kBlock), 0, s, a, b, cov, K, out, singular);
    return hipGetLastError();
}

// ------------------------------------------------------------- associate ---
// One wave walks the list 64 landmarks at a time; the first match (or the
// first singular covariance, where the reference raises) in list order wins.
__global__ __launch_bounds__(64) void k_associate(const double *obs, const double *lm, int32_t L,
                                                  double gate2, int32_t *out) {
    const int lane = threadIdx.x;
    const double ox = obs[0], oy = obs[1];
    for (int base = 0; base < L; base += 64) {
        const int j = base + lane;
        bool match = false, sing = false;
        if (j < L) {
            const double *s = lm + (int64_t)j * 6;
            M2 I;
            if (!inv2(M2{s[2], s[3], s[4], s[5]}, I)) {
                sing = true;
            } else {
                const double q = quad(I, ox - s[0], oy - s[1]);
                match = q >= 0.0 && q < gate2;
            }
        }
        const unsigned long long ev = __ballot(match || sing);
        if (ev) {
            const int first = __ffsll((long long)ev) - 1;
            if (lane == first) out[0] = sing ? -2 : j;
            return;
        }
    }
    if (lane == 0) out[0] = -1;
}

hipError_t launch_associate(const double *obs, const double *lm, int32_t L, double gate2,
                            int32_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_associate, dim3(1), dim3(64), 0, s, obs, lm, L, gate2, out);
    return hipGetLastError();
}

}  // namespace fs2
