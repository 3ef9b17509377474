// fs2_cluster.hip -- exact DBSCAN on gfx950 for the known-landmark map
// (reference: GeometryUtils.cluster_points, fast_slam_2/utils/geometry_utils.py:26-62,
// sklearn DBSCAN; called by LandmarkUtils.update_known_landmarks,
// fast_slam_2/utils/landmark_utils.py:120-144, over every landmark of every particle).
//
// sklearn's result, restated as a deterministic function of the points:
//   neighbour(p, q)  <=>  fl(fl(dx*dx) + fl(dy*dy)) <= fl(eps*eps)   (p itself counts);
//   core(p)          <=>  |{q : neighbour(p, q)}| >= min_samples;
//   clusters         =   connected components of the core points under neighbour,
//                        numbered by their smallest core-point index;
//   border point     ->  the lowest-numbered cluster with a core point in reach,
//                        else noise (-1);
//   centre           =   numpy mean(axis=0) of the members in index order, i.e. a
//                        sequential sum divided by the count.
//
// MI355X mapping.  Points are bucketed into square cells of side eps/(2*sqrt 2)
// (a cell's diagonal is eps/2) by one radix sort of 64-bit cell keys (stable, so
// each cell lists its points in index order).  The exact neighbour predicate is
// only evaluated where geometry cannot decide: with the true bounding box of each
// cell's points, a cell entirely within eps of a point is counted whole, a cell
// entirely beyond eps is skipped (1e-12 relative margins on both tests).  A cell
// with >= min_samples points is core throughout (all its points are within eps of
// each other); the core points of one cell are one node of the component graph,
// joined to the 7x7 neighbouring cells by a lock-free union-find.  At N = 1e6
// particles x 500 landmarks (5e8 points in ~2000 dense cells) this is one sort,
// a few streaming passes and a per-cluster sequential sum.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <vector>

#include "fs2_reduce.hpp"

namespace fs2 {

constexpr int kNbr = 49;                         // 7x7 cells around a cell
constexpr double kInside = 1.0 - 1e-12;          // "entirely within eps" margin
constexpr double kOutside = 1.0 + 1e-12;         // "entirely beyond eps" margin

struct ClusterGeom {
    double x0, y0, ih, eps, eps2;                // origin, 1/cell side, eps, fl(eps*eps)
};

__device__ __forceinline__ uint64_t cell_key(int64_t cx, int64_t cy) {
    return ((uint64_t)cy << 32) | (uint64_t)cx;
}

__device__ __forceinline__ bool neighbour(double2 p, double2 q, double eps2) {
    const double dx = p.x - q.x, dy = p.y - q.y;
    return dx * dx + dy * dy <= eps2;
}

// largest / smallest distance from p to the box (x0, y0, x1, y1)
__device__ __forceinline__ double box_max_dist(double2 p, const double4 &b) {
    const double dx = fmax(fabs(p.x - b.x), fabs(p.x - b.z)), dy = fmax(fabs(p.y - b.y), fabs(p.y - b.w));
    return sqrt(dx * dx + dy * dy);
}
__device__ __forceinline__ double box_min_dist(double2 p, const double4 &b) {
    const double dx = fmax(fmax(b.x - p.x, p.x - b.z), 0.0), dy = fmax(fmax(b.y - p.y, p.y - b.w), 0.0);
    return sqrt(dx * dx + dy * dy);
}
__device__ __forceinline__ double boxes_max_dist(const double4 &a, const double4 &b) {
    const double dx = fmax(b.z - a.x, a.z - b.x), dy = fmax(b.w - a.y, a.w - b.y);
    return sqrt(dx * dx + dy * dy);
}
__device__ __forceinline__ double boxes_min_dist(const double4 &a, const double4 &b) {
    const double dx = fmax(fmax(b.x - a.z, a.x - b.z), 0.0), dy = fmax(fmax(b.y - a.w, a.y - b.w), 0.0);
    return sqrt(dx * dx + dy * dy);
}

// ---- 1. bounding box / finiteness ----
__global__ __launch_bounds__(kBlock) void k_cl_bbox(const double2 *pts, int64_t n, double *part) {
    __shared__ double lds[4][kBlock / 64];
    double mx = INFINITY, my = INFINITY, bad = 0.0, ext = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const double2 p = pts[i];
        if (!(isfinite(p.x) && isfinite(p.y))) bad = 1.0;
        mx = fmin(mx, p.x);
        my = fmin(my, p.y);
        ext = fmax(ext, fmax(fabs(p.x), fabs(p.y)));
    }
    double v[4] = {mx, my, -bad, -ext};
#pragma unroll
    for (int q = 0; q < 4; ++q)
        for (int o = 32; o > 0; o >>= 1) v[q] = fmin(v[q], __shfl_xor(v[q], o, 64));
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
        for (int q = 0; q < 4; ++q) lds[q][wid] = v[q];
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 0; q < 4; ++q) {
            double t = lds[q][0];
            for (int k = 1; k < kBlock / 64; ++k) t = fmin(t, lds[q][k]);
            part[blockIdx.x * 4 + q] = t;
        }
    }
}

// ---- 2. cell keys ----
__global__ __launch_bounds__(kBlock) void k_cl_keys(const double2 *pts, int64_t n, ClusterGeom g, uint64_t *key,
                                                    uint32_t *idx) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double2 p = pts[i];
    const int64_t cx = (int64_t)floor((p.x - g.x0) * g.ih), cy = (int64_t)floor((p.y - g.y0) * g.ih);
    key[i] = cell_key(cx, cy);
    idx[i] = (uint32_t)i;
}

// ---- 3. cells of the sorted order ----
__global__ __launch_bounds__(kBlock) void k_cl_heads(const uint64_t *skey, int64_t n, int32_t *head) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k < n) head[k] = (k == 0 || skey[k] != skey[k - 1]) ? 1 : 0;
}

// cid = inclusive scan of heads - 1
__global__ __launch_bounds__(kBlock) void k_cl_cells(const uint64_t *skey, int64_t n, int32_t *cid,
                                                     const int32_t *head, int32_t *cstart, uint64_t *ckey) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const int32_t c = cid[k] - 1;
    cid[k] = c;
    if (head[k]) {
        cstart[c] = (int32_t)k;
        ckey[c] = skey[k];
    }
    if (k == n - 1) cstart[c + 1] = (int32_t)n;
}

// one wave per cell: box of its points
__global__ __launch_bounds__(kBlock) void k_cl_boxes(const double2 *pts, const uint32_t *sidx, const int32_t *cstart,
                                                     int32_t C, double4 *cbox) {
    const int c = (int)(((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= C) return;
    double x0 = INFINITY, y0 = INFINITY, x1 = -INFINITY, y1 = -INFINITY;
    for (int k = cstart[c] + lane; k < cstart[c + 1]; k += 64) {
        const double2 p = pts[sidx[k]];
        x0 = fmin(x0, p.x);
        y0 = fmin(y0, p.y);
        x1 = fmax(x1, p.x);
        y1 = fmax(y1, p.y);
    }
    for (int o = 32; o > 0; o >>= 1) {
        x0 = fmin(x0, __shfl_xor(x0, o, 64));
        y0 = fmin(y0, __shfl_xor(y0, o, 64));
        x1 = fmax(x1, __shfl_xor(x1, o, 64));
        y1 = fmax(y1, __shfl_xor(y1, o, 64));
    }
    if (lane == 0) cbox[c] = make_double4(x0, y0, x1, y1);
}

// neighbouring cells (7x7) by binary search over the sorted cell keys; -1 = none
__global__ __launch_bounds__(kBlock) void k_cl_nbrs(const uint64_t *ckey, int32_t C, int32_t *nbr) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (int64_t)C * kNbr) return;
    const int c = (int)(t / kNbr), o = (int)(t % kNbr);
    const int64_t cx = (int64_t)(ckey[c] & 0xffffffffull) + (o % 7) - 3;
    const int64_t cy = (int64_t)(ckey[c] >> 32) + (o / 7) - 3;
    int32_t r = -1;
    if (cx >= 0 && cy >= 0) {
        const uint64_t want = cell_key(cx, cy);
        int lo = 0, hi = C;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (ckey[mid] < want) lo = mid + 1;
            else hi = mid;
        }
        if (lo < C && ckey[lo] == want) r = lo;
    }
    nbr[t] = r;
}

// ---- 4. core points ----
__global__ __launch_bounds__(kBlock) void k_cl_core(const double2 *pts, const uint32_t *sidx, const int32_t *cid,
                                                    const int32_t *cstart, const double4 *cbox, const int32_t *nbr,
                                                    int64_t n, ClusterGeom g, int64_t min_samples, uint8_t *core) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const int c = cid[k];
    const int64_t own = cstart[c + 1] - cstart[c];
    const double4 ob = cbox[c];
    const double ein = g.eps * kInside, eout = g.eps * kOutside;
    if (own >= min_samples && boxes_max_dist(ob, ob) <= ein) {   // all within eps of each other
        core[k] = 1;
        return;
    }
    const double2 p = pts[sidx[k]];
    int64_t cnt = 0;
    for (int o = 0; o < kNbr && cnt < min_samples; ++o) {
        const int b = nbr[(int64_t)c * kNbr + o];
        if (b < 0) continue;
        const double4 bb = cbox[b];
        const int64_t sz = cstart[b + 1] - cstart[b];
        if (box_max_dist(p, bb) <= ein) {
            cnt += sz;
        } else if (box_min_dist(p, bb) <= eout) {
            for (int q = cstart[b]; q < cstart[b + 1] && cnt < min_samples; ++q)
                cnt += neighbour(p, pts[sidx[q]], g.eps2) ? 1 : 0;
        }
    }
    core[k] = cnt >= min_samples ? 1 : 0;
}

// one wave per cell: first core point (sorted position; smallest index among the
// cell's cores since the sort is stable) and the box of its core points
__global__ __launch_bounds__(kBlock) void k_cl_cellcore(const int32_t *cstart, const uint8_t *core, int32_t C,
                                                        int32_t *first_core) {
    const int c = (int)(((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= C) return;
    int found = -1;
    for (int k0 = cstart[c]; k0 < cstart[c + 1] && found < 0; k0 += 64) {
        const int k = k0 + lane;
        const uint64_t m = __ballot(k < cstart[c + 1] && core[k]);
        if (m) found = k0 + __ffsll((unsigned long long)m) - 1;
    }
    if (lane == 0) first_core[c] = found;
}

// Device-scope loads: a plain load may hit a stale line in this CU's L1 while
// other CUs hook roots in L2 (the CAS below always sees the L2 value).
__device__ __forceinline__ int uf_load(int32_t *parent, int x) {
    return __hip_atomic_load(parent + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int uf_find(int32_t *parent, int x) {
    int p = uf_load(parent, x);
    while (p != x) {
        const int gp = uf_load(parent, p);
        if (gp != p) parent[x] = gp;    // path halving (benign race)
        x = p;
        p = gp;
    }
    return x;
}

__device__ __forceinline__ void uf_union(int32_t *parent, int a, int b) {
    while (true) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        // hook the larger root under the smaller
        if (atomicCAS(&parent[a], a, b) == a) return;
    }
}

// ---- 5. components of the core points (cells as nodes) ----
__global__ __launch_bounds__(kBlock) void k_cl_union(const double2 *pts, const uint32_t *sidx, const int32_t *cstart,
                                                     const double4 *cbox, const int32_t *nbr,
                                                     const int32_t *first_core, const uint8_t *core, int32_t C,
                                                     ClusterGeom g, int32_t *parent) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (int64_t)C * kNbr) return;
    const int a = (int)(t / kNbr);
    const int b = nbr[t];
    if (b <= a || first_core[a] < 0 || first_core[b] < 0) return;
    const double4 ba = cbox[a], bb = cbox[b];
    bool joined;
    if (boxes_max_dist(ba, bb) <= g.eps * kInside) {
        joined = true;
    } else if (boxes_min_dist(ba, bb) > g.eps * kOutside) {
        joined = false;
    } else {
        joined = false;
        for (int p = first_core[a]; p < cstart[a + 1] && !joined; ++p) {
            if (!core[p]) continue;
            const double2 pp = pts[sidx[p]];
            for (int q = first_core[b]; q < cstart[b + 1]; ++q)
                if (core[q] && neighbour(pp, pts[sidx[q]], g.eps2)) {
                    joined = true;
                    break;
                }
        }
    }
    if (joined) uf_union(parent, a, b);
}

// Read-only find into a separate array: a compressing find here would race with
// the other threads' path halving (a halving store landing after parent[c] = root
// leaves parent[c] at a non-root ancestor).
__global__ __launch_bounds__(kBlock) void k_cl_roots(const int32_t *parent, const int32_t *first_core,
                                                     const uint32_t *sidx, int32_t C, int32_t *root,
                                                     uint32_t *comp_min) {
    const int c = (int)((int64_t)blockIdx.x * kBlock + threadIdx.x);
    if (c >= C) return;
    int r = c;
    while (parent[r] != r) r = parent[r];
    root[c] = r;
    if (first_core[c] >= 0) atomicMin(&comp_min[r], sidx[first_core[c]]);
}

// roots with cores -> (comp_min, root) pairs for the numbering sort
__global__ __launch_bounds__(kBlock) void k_cl_rootlist(const int32_t *root, const uint32_t *comp_min, int32_t C,
                                                        uint32_t *rkey, int32_t *rval, int32_t *nroots) {
    const int c = (int)((int64_t)blockIdx.x * kBlock + threadIdx.x);
    if (c >= C) return;
    if (root[c] == c && comp_min[c] != 0xffffffffu) {
        const int s = atomicAdd(nroots, 1);
        rkey[s] = comp_min[c];
        rval[s] = c;
    }
}

__global__ __launch_bounds__(kBlock) void k_cl_number(const int32_t *sorted_roots, int32_t K, int32_t *root_label) {
    const int r = (int)((int64_t)blockIdx.x * kBlock + threadIdx.x);
    if (r < K) root_label[sorted_roots[r]] = r;
}

// cell label: the label of its component if it has core points, else -1
__global__ __launch_bounds__(kBlock) void k_cl_celllabel(const int32_t *root, const int32_t *first_core,
                                                         const int32_t *root_label, int32_t C, int32_t *clabel) {
    const int c = (int)((int64_t)blockIdx.x * kBlock + threadIdx.x);
    if (c >= C) return;
    clabel[c] = first_core[c] >= 0 ? root_label[root[c]] : -1;
}

// ---- 6. labels: core -> its cluster; border -> lowest cluster in reach ----
__global__ __launch_bounds__(kBlock) void k_cl_label(const double2 *pts, const uint32_t *sidx, const int32_t *cid,
                                                     const int32_t *cstart, const double4 *cbox, const int32_t *nbr,
                                                     const int32_t *first_core, const uint8_t *core,
                                                     const int32_t *clabel, int64_t n, ClusterGeom g,
                                                     int32_t *labels) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const int c = cid[k];
    int lab;
    if (core[k]) {
        lab = clabel[c];
    } else {
        const double2 p = pts[sidx[k]];
        lab = INT32_MAX;
        for (int o = 0; o < kNbr; ++o) {
            const int b = nbr[(int64_t)c * kNbr + o];
            if (b < 0 || first_core[b] < 0 || clabel[b] >= lab) continue;
            const double4 bb = cbox[b];
            bool reach = false;
            if (box_max_dist(p, bb) <= g.eps * kInside) {
                reach = true;
            } else if (box_min_dist(p, bb) <= g.eps * kOutside) {
                for (int q = first_core[b]; q < cstart[b + 1] && !reach; ++q)
                    reach = core[q] && neighbour(p, pts[sidx[q]], g.eps2);
            }
            if (reach) lab = clabel[b];
        }
        if (lab == INT32_MAX) lab = -1;
    }
    labels[sidx[k]] = lab;
}

// ---- 7. centres: members in index order, sequential sums (numpy mean axis 0) ----
__global__ __launch_bounds__(kBlock) void k_cl_lkeys(const int32_t *labels, int64_t n, int32_t K, uint32_t *lkey,
                                                     uint32_t *lidx) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int32_t l = labels[i];
    lkey[i] = l < 0 ? (uint32_t)K : (uint32_t)l;
    lidx[i] = (uint32_t)i;
}

// One wave per cluster: the wave loads 64 members at a time (the next chunk in
// flight) and lane order is replayed into one sequential sum.
__global__ __launch_bounds__(kBlock) void k_cl_centres(const double2 *pts, const uint32_t *slkey, const uint32_t *slidx,
                                                       int64_t n, int32_t K, double *centres) {
    const int l = (int)(((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (l >= K) return;
    auto first_of = [&](uint32_t v) {
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (slkey[mid] < v) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const int64_t lo = first_of((uint32_t)l), hi = first_of((uint32_t)l + 1u);
    double sx = 0.0, sy = 0.0;
    double2 cur = (lo + lane < hi) ? pts[slidx[lo + lane]] : make_double2(0.0, 0.0);
    for (int64_t k0 = lo; k0 < hi; k0 += 64) {
        const int64_t kn = k0 + 64 + lane;
        const double2 nxt = (kn < hi) ? pts[slidx[kn]] : make_double2(0.0, 0.0);
        const int m = (int)std::min<int64_t>(64, hi - k0);
        for (int u = 0; u < m; ++u) {
            sx += __shfl(cur.x, u, 64);
            sy += __shfl(cur.y, u, 64);
        }
        cur = nxt;
    }
    if (lane == 0) {
        const double cnt = (double)(hi - lo);
        centres[2 * l] = sx / cnt;
        centres[2 * l + 1] = sy / cnt;
    }
}

__global__ void k_cl_iota(int32_t *p, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t < n) p[t] = (int32_t)t;
}

__global__ void k_cl_widen(const int32_t *a, int64_t n, int64_t *b) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t < n) b[t] = a[t];
}

// ---- driver ----

#define CL_TRY(expr)                                    \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return e_;                \
    } while (0)

static unsigned cl_grid(int64_t total) { return (unsigned)((total + kBlock - 1) / kBlock); }

// Scratch owned by one call, released on return.
struct ClusterScratch {
    std::vector<void *> ptrs;
    ~ClusterScratch() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    hipError_t get(T **out, size_t count) {
        void *p = nullptr;
        hipError_t e = hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) ptrs.push_back(p);
        *out = static_cast<T *>(p);
        return e;
    }
};

hipError_t cluster_points(const double2 *pts, int64_t n, double eps, int64_t min_samples, double *centres_out,
                          int64_t centres_cap, int64_t *nclusters, int32_t *labels_out, int32_t *status,
                          hipStream_t s) {
    *status = 0;
    *nclusters = 0;
    ClusterScratch sc;
    // bbox + finiteness
    const unsigned gb = std::min<unsigned>(cl_grid(n), 1024u);
    double *part;
    CL_TRY(sc.get(&part, (size_t)gb * 4));
    hipLaunchKernelGGL(k_cl_bbox, dim3(gb), dim3(kBlock), 0, s, pts, n, part);
    std::vector<double> hp((size_t)gb * 4);
    CL_TRY(hipMemcpyAsync(hp.data(), part, hp.size() * 8, hipMemcpyDeviceToHost, s));
    CL_TRY(hipStreamSynchronize(s));
    double mx = INFINITY, my = INFINITY, bad = 0.0, ext = 0.0;
    for (unsigned b = 0; b < gb; ++b) {
        mx = std::min(mx, hp[b * 4]);
        my = std::min(my, hp[b * 4 + 1]);
        bad = std::min(bad, hp[b * 4 + 2]);
        ext = std::min(ext, hp[b * 4 + 3]);
    }
    if (bad < 0.0) {
        *status = 1;                  // sklearn: "Input contains NaN or infinity"
        return hipSuccess;
    }
    ClusterGeom g;
    g.x0 = mx;
    g.y0 = my;
    g.eps = eps;
    g.eps2 = eps * eps;
    g.ih = 1.0 / (eps * 0.35355339059327373);     // cell side eps / (2 sqrt 2)
    if (2.0 * (-ext) * g.ih > 2.0e9) {
        *status = 2;                  // coordinate span too large for 32-bit cell indices
        return hipSuccess;
    }
    // sort points by cell (stable: index order inside a cell)
    uint64_t *key, *skey;
    uint32_t *idx, *sidx;
    CL_TRY(sc.get(&key, n));
    CL_TRY(sc.get(&skey, n));
    CL_TRY(sc.get(&idx, n));
    CL_TRY(sc.get(&sidx, n));
    hipLaunchKernelGGL(k_cl_keys, dim3(cl_grid(n)), dim3(kBlock), 0, s, pts, n, g, key, idx);
    const double span = 2.0 * (-ext) * g.ih + 2.0;
    unsigned bits = 1;
    while (bits < 32 && (double)(1ull << bits) <= span) ++bits;
    size_t tmp_bytes = 0;
    CL_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, key, skey, idx, sidx, (size_t)n, 0, 32 + bits, s));
    void *tmp;
    CL_TRY(sc.get((char **)&tmp, tmp_bytes));
    // cells on the x axis use bits [0, bits), on the y axis [32, 32 + bits)
    CL_TRY(rocprim::radix_sort_pairs(tmp, tmp_bytes, key, skey, idx, sidx, (size_t)n, 0, 32 + bits, s));
    int32_t *head, *cid;
    CL_TRY(sc.get(&head, n));
    CL_TRY(sc.get(&cid, n));
    hipLaunchKernelGGL(k_cl_heads, dim3(cl_grid(n)), dim3(kBlock), 0, s, skey, n, head);
    size_t scan_bytes = 0;
    CL_TRY(rocprim::inclusive_scan(nullptr, scan_bytes, head, cid, (size_t)n, rocprim::plus<int32_t>(), s));
    void *stmp;
    CL_TRY(sc.get((char **)&stmp, scan_bytes));
    CL_TRY(rocprim::inclusive_scan(stmp, scan_bytes, head, cid, (size_t)n, rocprim::plus<int32_t>(), s));
    int32_t C = 0;
    CL_TRY(hipMemcpyAsync(&C, cid + n - 1, 4, hipMemcpyDeviceToHost, s));
    CL_TRY(hipStreamSynchronize(s));
    int32_t *cstart, *nbr, *first_core, *parent, *root, *clabel, *root_label, *rval, *srval, *nroots;
    uint64_t *ckey;
    double4 *cbox;
    uint32_t *comp_min, *rkey, *srkey;
    uint8_t *core;
    CL_TRY(sc.get(&cstart, (size_t)C + 1));
    CL_TRY(sc.get(&ckey, C));
    CL_TRY(sc.get(&cbox, C));
    CL_TRY(sc.get(&nbr, (size_t)C * kNbr));
    CL_TRY(sc.get(&core, n));
    CL_TRY(sc.get(&first_core, C));
    CL_TRY(sc.get(&parent, C));
    CL_TRY(sc.get(&root, C));
    CL_TRY(sc.get(&comp_min, C));
    CL_TRY(sc.get(&clabel, C));
    CL_TRY(sc.get(&root_label, C));
    CL_TRY(sc.get(&rkey, C));
    CL_TRY(sc.get(&srkey, C));
    CL_TRY(sc.get(&rval, C));
    CL_TRY(sc.get(&srval, C));
    CL_TRY(sc.get(&nroots, 1));
    hipLaunchKernelGGL(k_cl_cells, dim3(cl_grid(n)), dim3(kBlock), 0, s, skey, n, cid, head, cstart, ckey);
    hipLaunchKernelGGL(k_cl_boxes, dim3(cl_grid((int64_t)C * 64)), dim3(kBlock), 0, s, pts, sidx, cstart, C, cbox);
    hipLaunchKernelGGL(k_cl_nbrs, dim3(cl_grid((int64_t)C * kNbr)), dim3(kBlock), 0, s, ckey, C, nbr);
    hipLaunchKernelGGL(k_cl_core, dim3(cl_grid(n)), dim3(kBlock), 0, s, pts, sidx, cid, cstart, cbox, nbr, n, g,
                       min_samples, core);
    hipLaunchKernelGGL(k_cl_cellcore, dim3(cl_grid((int64_t)C * 64)), dim3(kBlock), 0, s, cstart, core, C,
                       first_core);
    hipLaunchKernelGGL(k_cl_iota, dim3(cl_grid(C)), dim3(kBlock), 0, s, parent, (int64_t)C);
    CL_TRY(hipMemsetAsync(comp_min, 0xff, sizeof(uint32_t) * C, s));
    CL_TRY(hipMemsetAsync(nroots, 0, 4, s));
    hipLaunchKernelGGL(k_cl_union, dim3(cl_grid((int64_t)C * kNbr)), dim3(kBlock), 0, s, pts, sidx, cstart, cbox, nbr,
                       first_core, core, C, g, parent);
    hipLaunchKernelGGL(k_cl_roots, dim3(cl_grid(C)), dim3(kBlock), 0, s, parent, first_core, sidx, C, root,
                       comp_min);
    hipLaunchKernelGGL(k_cl_rootlist, dim3(cl_grid(C)), dim3(kBlock), 0, s, root, comp_min, C, rkey, rval, nroots);
    int32_t K = 0;
    CL_TRY(hipMemcpyAsync(&K, nroots, 4, hipMemcpyDeviceToHost, s));
    CL_TRY(hipStreamSynchronize(s));
    if (K > 0) {
        size_t rb = 0;
        CL_TRY(rocprim::radix_sort_pairs(nullptr, rb, rkey, srkey, rval, srval, (size_t)K, 0, 32, s));
        void *rtmp;
        CL_TRY(sc.get((char **)&rtmp, rb));
        CL_TRY(rocprim::radix_sort_pairs(rtmp, rb, rkey, srkey, rval, srval, (size_t)K, 0, 32, s));
        hipLaunchKernelGGL(k_cl_number, dim3(cl_grid(K)), dim3(kBlock), 0, s, srval, K, root_label);
    }
    hipLaunchKernelGGL(k_cl_celllabel, dim3(cl_grid(C)), dim3(kBlock), 0, s, root, first_core, root_label, C,
                       clabel);
    int32_t *labels;
    CL_TRY(sc.get(&labels, n));
    hipLaunchKernelGGL(k_cl_label, dim3(cl_grid(n)), dim3(kBlock), 0, s, pts, sidx, cid, cstart, cbox, nbr,
                       first_core, core, clabel, n, g, labels);
    *nclusters = K;
    if (labels_out) CL_TRY(hipMemcpyAsync(labels_out, labels, sizeof(int32_t) * n, hipMemcpyDefault, s));
    if (K > 0 && centres_out && centres_cap >= K) {
        // members of each cluster in index order (stable sort by label)
        uint32_t *lkey = reinterpret_cast<uint32_t *>(key), *lidx = idx;     // reuse
        uint32_t *slkey = reinterpret_cast<uint32_t *>(skey), *slidx = sidx;
        hipLaunchKernelGGL(k_cl_lkeys, dim3(cl_grid(n)), dim3(kBlock), 0, s, labels, n, K, lkey, lidx);
        size_t lb = 0;
        unsigned lbits = 1;
        while (lbits < 32 && (1ll << lbits) <= (int64_t)K) ++lbits;
        CL_TRY(rocprim::radix_sort_pairs(nullptr, lb, lkey, slkey, lidx, slidx, (size_t)n, 0, lbits, s));
        void *ltmp;
        CL_TRY(sc.get((char **)&ltmp, lb));
        CL_TRY(rocprim::radix_sort_pairs(ltmp, lb, lkey, slkey, lidx, slidx, (size_t)n, 0, lbits, s));
        double *dcent;
        CL_TRY(sc.get(&dcent, (size_t)K * 2));
        hipLaunchKernelGGL(k_cl_centres, dim3(cl_grid((int64_t)K * 64)), dim3(kBlock), 0, s, pts, slkey, slidx, n,
                           K, dcent);
        CL_TRY(hipMemcpyAsync(centres_out, dcent, sizeof(double) * 2 * K, hipMemcpyDefault, s));
    }
    CL_TRY(hipStreamSynchronize(s));
    return hipGetLastError();
}

// Landmarks of particles [0, n) in (particle, slot) order -> points (x, y); one
// thread per (page row, particle), rows outer so a wave reads one page-table row.
__global__ __launch_bounds__(kBlock) void k_cl_gather_maps(MapRef map, const int32_t *cnt, const int64_t *off,
                                                           int64_t n, double2 *out) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (int64_t)map.rows * n) return;
    const int row = (int)(t / n);
    const int64_t i = t % n;
    const int c = cnt[i];
    const int j0 = row * kPageSlots;
    if (j0 >= c) return;
    const uint32_t e = *pt_entry(map, row, i);
    const char *pg = page_ptr_any(map, e), *recs = recs_of(map, e);    // (a remote page: its rank's pools)
    double2 *o = out + off[i];
    for (int j = j0; j < min(c, j0 + kPageSlots); ++j) {      // position j holds slot mirror_slot
        const float4 mv = load_mirror(pg, j);
        const Slot sl = load_rec(recs, mirror_rec(mv));
        o[mirror_slot(mv)] = make_double2(sl.mx, sl.my);
    }
}

hipError_t gather_map_points(MapRef map, const int32_t *cnt, int64_t n, double2 **pts_out, int64_t *npts,
                             hipStream_t s) {
    *pts_out = nullptr;
    *npts = 0;
    if (n <= 0) return hipSuccess;
    ClusterScratch sc;
    int64_t *off, *c64;
    CL_TRY(sc.get(&off, n + 1));
    CL_TRY(sc.get(&c64, n));
    hipLaunchKernelGGL(k_cl_widen, dim3(cl_grid(n)), dim3(kBlock), 0, s, cnt, n, c64);
    size_t sb = 0;
    CL_TRY(rocprim::exclusive_scan(nullptr, sb, c64, off, (int64_t)0, (size_t)n, rocprim::plus<int64_t>(), s));
    void *stmp;
    CL_TRY(sc.get((char **)&stmp, sb));
    CL_TRY(rocprim::exclusive_scan(stmp, sb, c64, off, (int64_t)0, (size_t)n, rocprim::plus<int64_t>(), s));
    int64_t base = 0;
    int32_t last = 0;
    CL_TRY(hipMemcpyAsync(&base, off + n - 1, 8, hipMemcpyDeviceToHost, s));
    CL_TRY(hipMemcpyAsync(&last, cnt + n - 1, 4, hipMemcpyDeviceToHost, s));
    CL_TRY(hipStreamSynchronize(s));
    const int64_t total = base + last;
    double2 *pts = nullptr;
    CL_TRY(hipMalloc(&pts, sizeof(double2) * std::max<int64_t>(total, 1)));
    hipLaunchKernelGGL(k_cl_gather_maps, dim3(cl_grid((int64_t)map.rows * n)), dim3(kBlock), 0, s, map, cnt, off, n,
                       pts);
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        (void)hipFree(pts);
        return e;
    }
    *pts_out = pts;
    *npts = total;
    return hipGetLastError();
}

}  // namespace fs2
