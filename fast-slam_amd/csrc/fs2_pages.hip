// fs2_pages.hip -- collection of the landmark page pool.
//
// Pages are shared between particles after a resample and copied on their
// first write, so a page becomes garbage when the last page-table entry that
// refers to it is overwritten (a copy-on-write, a dropped particle, an import).
// Nothing counts references on the hot path; instead, when the host runs out
// of reserved free pages, it collects: mark every page the live page table
// refers to, then list every unmarked page as free.  Allocation between two
// collections is a cursor into that list (PageAlloc), so no kernel takes a
// lock or an atomic to get a page.
//
//   k_mark        one lane per particle, one byte store per page of its map
//   k_sweep_count free pages per 4096-page block
//   k_sweep_scan  exclusive scan of the block counts (one workgroup, 8192-count tiles)
//   k_sweep_write free page ids, in id order, into freel (staged in LDS, stored contiguously)
//
// Slot records (fs2_kernels.hpp) are collected the same way, less often (the
// record pool is sized for many scans of writes): after the page mark, every
// marked page marks the records its 8 mirrors name (k_mark_recs), and the same
// sweep lists the unmarked records.  A mirror past the map's end (in the last,
// partly filled page) may name a stale record; it is marked too, which only
// keeps that record out of the free list until the slot is overwritten.
#include "fs2_reduce.hpp"

namespace fs2 {

constexpr int kSweepPer = 16;                        // page ids per thread
constexpr int kSweepBlock = kBlock * kSweepPer;      // page ids per workgroup

int64_t collect_blocks(int64_t npool) { return (npool + kSweepBlock - 1) / kSweepBlock; }

// One lane per particle; its page-table entries are loaded 8 at a time (a mark
// store may alias them, so one load per iteration would pay a full memory
// latency per row).
// page_refs mode (map.peers, epochs: every rank's epoch of this collective
// collection): a remote page is marked in its owner's marks.
__global__ __launch_bounds__(kBlock) void k_mark(const MapRef map, const int32_t *cnt, uint8_t *mark,
                                                 uint8_t epoch, const uint8_t *epochs) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= map.n) return;
    const int rows = (cnt[i] + kPageSlots - 1) / kPageSlots;
    bool remote = false;
    for (int r0 = 0; r0 < rows; r0 += 8) {
        uint32_t e[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) e[u] = *pt_entry(map, min(r0 + u, rows - 1), i);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (r0 + u >= rows) continue;
            const uint32_t t = map.peers ? ref_tag(e[u]) : 0u;
            if (t) {
                map.peers->mark[t - 1][ref_id(e[u])] = epochs[t - 1];
                remote = true;
            } else {
                mark[e[u] & kIdMask] = epoch;
            }
        }
    }
    // marks in other ranks' memory reach it before this rank's barrier
    if (__any(remote)) __threadfence_system();
}

__device__ __forceinline__ int wave_incl_scan_int(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// exclusive prefix of v over the workgroup (kBlock threads); total in *tot
__device__ __forceinline__ int block_excl_scan(int v, int *lds, int *tot) {
    const int inc = wave_incl_scan_int(v);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) lds[wid] = inc;
    __syncthreads();
    int off = 0, t = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
        if (k < wid) off += lds[k];
        t += lds[k];
    }
    *tot = t;
    return off + inc - v;
}

// free ids among the kSweepPer consecutive ids from id0 (bit e: id0 + e), from
// one 16-byte load of their marks; ids past npool are not free
__device__ __forceinline__ unsigned free_bits(const uint8_t *mark, int64_t npool, uint8_t epoch,
                                              int64_t id0) {
    unsigned bits = 0;
    if (id0 + kSweepPer <= npool) {
        const uint4 v = *reinterpret_cast<const uint4 *>(mark + id0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (((w[q] >> (8 * b)) & 0xffu) != epoch) bits |= 1u << (4 * q + b);
    } else {
        for (int e = 0; e < kSweepPer; ++e)
            if (id0 + e < npool && mark[id0 + e] != epoch) bits |= 1u << e;
    }
    return bits;
}

__global__ __launch_bounds__(kBlock) void k_sweep_count(const uint8_t *mark, int64_t npool, uint8_t epoch,
                                                        int64_t *bcnt) {
    __shared__ int lds[kBlock / 64];
    const int64_t id0 = (int64_t)blockIdx.x * kSweepBlock + (int64_t)threadIdx.x * kSweepPer;
    const int f = __popc(free_bits(mark, npool, epoch, id0));
    int tot;
    block_excl_scan(f, lds, &tot);
    if (threadIdx.x == 0) bcnt[blockIdx.x] = tot;
}

// exclusive scan of the block counts in place; *nfree = total.  Tiles of
// 1024 x 8 counts: each thread loads 8 consecutive counts of the tile at once
// (independent loads, one memory latency per tile), the workgroup scans their
// sums, and a running carry joins the tiles.
constexpr int kScanPer = 8;
__global__ __launch_bounds__(1024) void k_sweep_scan(int64_t *bcnt, int64_t nb, int64_t *nfree) {
    __shared__ int64_t lds[1024 / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t carry = 0;
    for (int64_t base = 0; base < nb; base += 1024 * kScanPer) {
        const int64_t b0 = base + (int64_t)threadIdx.x * kScanPer;
        int64_t c[kScanPer];
        int64_t s = 0;
#pragma unroll
        for (int u = 0; u < kScanPer; ++u) {
            c[u] = (b0 + u < nb) ? bcnt[b0 + u] : 0;
            s += c[u];
        }
        // inclusive scan of the per-thread sums
        int64_t v = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_up(v, d, 64);
            if (lane >= d) v += o;
        }
        if (lane == 63) lds[wid] = v;
        __syncthreads();
        int64_t off = 0, tot = 0;
        for (int k = 0; k < 1024 / 64; ++k) {
            if (k < wid) off += lds[k];
            tot += lds[k];
        }
        int64_t run = carry + off + v - s;
#pragma unroll
        for (int u = 0; u < kScanPer; ++u) {
            if (b0 + u < nb) bcnt[b0 + u] = run;
            run += c[u];
        }
        carry += tot;
        __syncthreads();                  // lds is rewritten by the next tile
    }
    if (threadIdx.x == 0) *nfree = carry;
}

// The workgroup's free ids, in id order, staged in LDS and stored contiguously
// (a lane storing its own run of ids would scatter 4-byte stores).
__global__ __launch_bounds__(kBlock) void k_sweep_write(const uint8_t *mark, int64_t npool, uint8_t epoch,
                                                        const int64_t *bcnt, uint32_t *freel) {
    __shared__ int lds[kBlock / 64];
    __shared__ uint32_t s_ids[kSweepBlock];
    const int64_t id0 = (int64_t)blockIdx.x * kSweepBlock + (int64_t)threadIdx.x * kSweepPer;
    unsigned bits = free_bits(mark, npool, epoch, id0);
    int tot;
    int pos = block_excl_scan(__popc(bits), lds, &tot);
    while (bits) {
        const int e = __builtin_ctz(bits);
        bits &= bits - 1u;
        s_ids[pos++] = (uint32_t)(id0 + e);
    }
    __syncthreads();
    uint32_t *dst = freel + bcnt[blockIdx.x];
    for (int j = threadIdx.x; j < tot; j += kBlock) dst[j] = s_ids[j];
}

// 8 consecutive lanes per page of the pool, each reading one 16-byte mirror of
// the page (one 128-byte line per 8 lanes).  A fixed grid strides over the pool,
// kMarkRecsAhead items per lane with their mark bytes loaded together: most pages
// are unmarked, and a one-item lane per (page, slot) needed npool/32 workgroups
// whose dispatch, not the bytes, set the kernel's time.
constexpr int kMarkRecsAhead = 4;
constexpr unsigned kMarkRecsGrid = 4096;
__global__ __launch_bounds__(kBlock) void k_mark_recs(const char *pool, int64_t npool, const uint8_t *mark,
                                                      uint8_t epoch, int64_t nrecs, uint8_t *rmark,
                                                      uint8_t repoch) {
    const int64_t lanes = npool * kPageSlots;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; t0 < lanes; t0 += kMarkRecsAhead * stride) {
        bool live[kMarkRecsAhead];
#pragma unroll
        for (int u = 0; u < kMarkRecsAhead; ++u) {
            const int64_t t = t0 + u * stride;
            live[u] = t < lanes && mark[t / kPageSlots] == epoch;
        }
        uint32_t r[kMarkRecsAhead];
#pragma unroll
        for (int u = 0; u < kMarkRecsAhead; ++u) {
            const int64_t t = t0 + u * stride;
            r[u] = live[u] ? mirror_rec(load_mirror(pool + (t / kPageSlots) * kPageBytes, (int)(t % kPageSlots)))
                           : 0xffffffffu;
        }
#pragma unroll
        for (int u = 0; u < kMarkRecsAhead; ++u)
            if (live[u] && (int64_t)r[u] < nrecs) rmark[r[u]] = repoch;
    }
}

hipError_t launch_collect_records(const char *pool, int64_t npool, const uint8_t *mark, uint8_t epoch,
                                  int64_t nrecs, uint8_t *rmark, uint8_t repoch, int64_t *rbcnt,
                                  uint32_t *rfreel, int64_t *rnfree_dev, hipStream_t s) {
    const int64_t nb = collect_blocks(nrecs);
    const int64_t lanes = npool * kPageSlots;
    if (lanes > 0) {
        const int64_t grid = std::min<int64_t>((lanes + kBlock - 1) / kBlock, kMarkRecsGrid);
        hipLaunchKernelGGL(k_mark_recs, dim3((unsigned)grid), dim3(kBlock), 0, s, pool, npool, mark, epoch, nrecs,
                           rmark, repoch);
    }
    hipLaunchKernelGGL(k_sweep_count, dim3((unsigned)nb), dim3(kBlock), 0, s, rmark, nrecs, repoch, rbcnt);
    hipLaunchKernelGGL(k_sweep_scan, dim3(1), dim3(1024), 0, s, rbcnt, nb, rnfree_dev);
    hipLaunchKernelGGL(k_sweep_write, dim3((unsigned)nb), dim3(kBlock), 0, s, rmark, nrecs, repoch, rbcnt, rfreel);
    return hipGetLastError();
}

hipError_t launch_collect_mark(MapRef map, const int32_t *cnt, uint8_t *mark, uint8_t epoch, const uint8_t *epochs,
                               hipStream_t s) {
    if (map.n > 0)
        hipLaunchKernelGGL(k_mark, dim3((unsigned)((map.n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, map,
                           cnt, mark, epoch, epochs);
    return hipGetLastError();
}

hipError_t launch_collect_sweep(int64_t npool, uint8_t *mark, uint8_t epoch, int64_t *bcnt, uint32_t *freel,
                                int64_t *nfree_dev, hipStream_t s) {
    const int64_t nb = collect_blocks(npool);
    hipLaunchKernelGGL(k_sweep_count, dim3((unsigned)nb), dim3(kBlock), 0, s, mark, npool, epoch, bcnt);
    hipLaunchKernelGGL(k_sweep_scan, dim3(1), dim3(1024), 0, s, bcnt, nb, nfree_dev);
    hipLaunchKernelGGL(k_sweep_write, dim3((unsigned)nb), dim3(kBlock), 0, s, mark, npool, epoch, bcnt, freel);
    return hipGetLastError();
}

hipError_t launch_collect(MapRef map, const int32_t *cnt, int64_t npool, uint8_t *mark, uint8_t epoch,
                          int64_t *bcnt, uint32_t *freel, int64_t *nfree_dev, hipStream_t s) {
    const int64_t nb = collect_blocks(npool);
    if (map.n > 0)
        hipLaunchKernelGGL(k_mark, dim3((unsigned)((map.n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, map,
                           cnt, mark, epoch, nullptr);
    hipLaunchKernelGGL(k_sweep_count, dim3((unsigned)nb), dim3(kBlock), 0, s, mark, npool, epoch, bcnt);
    hipLaunchKernelGGL(k_sweep_scan, dim3(1), dim3(1024), 0, s, bcnt, nb, nfree_dev);
    hipLaunchKernelGGL(k_sweep_write, dim3((unsigned)nb), dim3(kBlock), 0, s, mark, npool, epoch, bcnt, freel);
    return hipGetLastError();
}

}  // namespace fs2

#ifdef FS2_TEST_HOOKS
// Test hook (tests/test_gpu_parity.py, a separate libfs2_hooks.so built from this
// file alone): k_sweep_scan on host counts, for block counts past one tile.
extern "C" int fs2_debug_sweep_scan(int32_t device, int64_t *counts, int64_t nb, int64_t *total) {
    if (hipSetDevice(device) != hipSuccess) return -2;
    int64_t *d = nullptr;
    if (hipMalloc(&d, sizeof(int64_t) * (size_t)(nb + 1)) != hipSuccess) return -3;
    hipError_t e = hipMemcpy(d, counts, sizeof(int64_t) * (size_t)nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(fs2::k_sweep_scan, dim3(1), dim3(1024), 0, 0, d, nb, d + nb);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(counts, d, sizeof(int64_t) * (size_t)nb, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(total, d + nb, sizeof(int64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? 0 : -2;
}
#endif
