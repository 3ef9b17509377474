// ubench_gather.hip -- the resample's page-table row copy on gfx950 (what
// k_gather_rows does: output m takes source s(m)'s row entries, column-major
// tables of 8-byte descriptors [rows][n], n = 10^6, 63 rows, sources from a
// systematic resample of lognormal weights, non-decreasing, N_eff / N ~ 0.45).
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_gather scripts/ubench_gather.hip
//   scripts/ubench_gather
//
// Variants (time per copy, GB/s of the 2 x 8 B x rows x n algorithmic bytes):
//   g8nt     tasks (output block, 8 rows), 8 entries in flight per lane, nt stores (libfs2)
//   g8       the same, plain stores
//   g16nt    16 rows per task
//   ident    g8nt with s(m) = m (a streaming copy: the layout's ceiling)
//   loop     one lane per output walking all rows, 8 per round (round 4's fused loop)
//   pair     two outputs per lane, 16-byte stores (1 KB per wave and row)
//   rowmaj   one workgroup per row-group slab: blockIdx = (row group, output block), row group slowest
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

typedef unsigned long long u64;

template <int RG, bool NT>
__global__ __launch_bounds__(256) void k_tasks(const u64 *A, u64 *B, const int *src, int64_t n, int rows, int slow_rows) {
    const int64_t nob = (n + 255) / 256;
    const int64_t ng = (rows + RG - 1) / RG;
    const int64_t tasks = nob * ng;
    for (int64_t t = blockIdx.x; t < tasks; t += gridDim.x) {
        const int64_t b = slow_rows ? t / ng : t % nob;
        const int k0 = (int)(slow_rows ? t % ng : t / nob) * RG;
        const int64_t m = b * 256 + threadIdx.x;
        if (m >= n) continue;
        const int s = src[m];
        u64 e[RG];
#pragma unroll
        for (int u = 0; u < RG; ++u) e[u] = A[(int64_t)std::min(k0 + u, rows - 1) * n + s];
#pragma unroll
        for (int u = 0; u < RG; ++u)
            if (k0 + u < rows) {
                u64 *d = B + (int64_t)(k0 + u) * n + m;
                if (NT) __builtin_nontemporal_store(e[u], d);
                else *d = e[u];
            }
    }
}

__global__ __launch_bounds__(256) void k_loop(const u64 *A, u64 *B, const int *src, int64_t n, int rows) {
    const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (m >= n) return;
    const int s = src[m];
    for (int k0 = 0; k0 < rows; k0 += 8) {
        u64 e[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) e[u] = A[(int64_t)std::min(k0 + u, rows - 1) * n + s];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (k0 + u < rows) __builtin_nontemporal_store(e[u], B + (int64_t)(k0 + u) * n + m);
    }
}

typedef u64 u64x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_pair(const u64 *A, u64 *B, const int *src, int64_t n, int rows) {
    const int64_t nob = (n + 511) / 512;
    const int64_t ng = (rows + 7) / 8;
    const int64_t tasks = nob * ng;
    for (int64_t t = blockIdx.x; t < tasks; t += gridDim.x) {
        const int64_t b = t % nob;
        const int k0 = (int)(t / nob) * 8;
        const int64_t m = b * 512 + 2 * threadIdx.x;
        if (m + 1 >= n) continue;
        const int s0 = src[m], s1 = src[m + 1];
        u64 e0[8], e1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t r = (int64_t)std::min(k0 + u, rows - 1) * n;
            e0[u] = A[r + s0];
            e1[u] = A[r + s1];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (k0 + u < rows) {
                u64x2 v;
                v.x = e0[u];
                v.y = e1[u];
                __builtin_nontemporal_store(v, reinterpret_cast<u64x2 *>(B + (int64_t)(k0 + u) * n + m));
            }
    }
}

int main() {
    const int64_t n = 1000000;
    const int rows = 63;
    std::vector<int> hs(n), hid(n);
    {
        std::mt19937_64 g(1);
        std::lognormal_distribution<double> ln(0.0, std::sqrt(-std::log(0.45)));
        std::vector<double> w(n), c(n);
        double t = 0;
        for (int64_t i = 0; i < n; ++i) t += (w[i] = ln(g));
        double a = 0;
        for (int64_t i = 0; i < n; ++i) c[i] = (a += w[i] / t);
        const double u0 = std::uniform_real_distribution<double>(0, 1.0 / n)(g);
        int64_t j = 0;
        int64_t distinct = 0;
        for (int64_t m = 0; m < n; ++m) {
            const double u = u0 + (double)m / n;
            while (j < n - 1 && u > c[j]) ++j;
            hs[m] = (int)j;
            distinct += (m == 0 || hs[m] != hs[m - 1]);
            hid[m] = (int)m;
        }
        std::printf("sources: %lld distinct of %lld\n", (long long)distinct, (long long)n);
    }
    u64 *A, *B;
    int *src, *ident;
    const size_t tb = sizeof(u64) * (size_t)rows * n;
    CK(hipMalloc(&A, tb));
    CK(hipMalloc(&B, tb));
    CK(hipMalloc(&src, 4 * n));
    CK(hipMalloc(&ident, 4 * n));
    CK(hipMemset(A, 1, tb));
    CK(hipMemset(B, 0, tb));
    CK(hipMemcpy(src, hs.data(), 4 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(ident, hid.data(), 4 * n, hipMemcpyHostToDevice));
    // a scratch buffer swept between reps: the tables start cold as after a scan
    char *scratch;
    const size_t sb = 1ull << 30;
    CK(hipMalloc(&scratch, sb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int64_t nob = (n + 255) / 256;
    auto run = [&](const char *name, auto launch) {
        float best = 1e9f, sum = 0.f;
        const int reps = 7;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemsetAsync(scratch, r, sb));
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
            sum += ms;
        }
        const double bytes = 2.0 * 8.0 * rows * n;
        std::printf("%-8s best %7.1f us  mean %7.1f us  %6.0f GB/s (best)\n", name, best * 1e3, sum / reps * 1e3,
                    bytes / (best * 1e-3) / 1e9);
    };
    const unsigned grid = 4096;
    run("g8nt", [&] { hipLaunchKernelGGL((k_tasks<8, true>), dim3(grid), dim3(256), 0, 0, A, B, src, n, rows, 0); });
    run("g8", [&] { hipLaunchKernelGGL((k_tasks<8, false>), dim3(grid), dim3(256), 0, 0, A, B, src, n, rows, 0); });
    run("g16nt", [&] { hipLaunchKernelGGL((k_tasks<16, true>), dim3(grid), dim3(256), 0, 0, A, B, src, n, rows, 0); });
    run("g4nt", [&] { hipLaunchKernelGGL((k_tasks<4, true>), dim3(grid), dim3(256), 0, 0, A, B, src, n, rows, 0); });
    run("g8full", [&] {
        hipLaunchKernelGGL((k_tasks<8, true>), dim3((unsigned)(nob * 8)), dim3(256), 0, 0, A, B, src, n, rows, 0);
    });
    run("ident", [&] { hipLaunchKernelGGL((k_tasks<8, true>), dim3(grid), dim3(256), 0, 0, A, B, ident, n, rows, 0); });
    run("identpl", [&] { hipLaunchKernelGGL((k_tasks<8, false>), dim3(grid), dim3(256), 0, 0, A, B, ident, n, rows, 0); });
    run("loop", [&] { hipLaunchKernelGGL(k_loop, dim3((unsigned)nob), dim3(256), 0, 0, A, B, src, n, rows); });
    run("pair", [&] { hipLaunchKernelGGL(k_pair, dim3(grid), dim3(256), 0, 0, A, B, src, n, rows); });
    run("rowmaj", [&] { hipLaunchKernelGGL((k_tasks<8, true>), dim3(grid), dim3(256), 0, 0, A, B, src, n, rows, 1); });
    run("memcpy", [&] { CK(hipMemcpyAsync(B, A, tb, hipMemcpyDeviceToDevice)); });
    return 0;
}
